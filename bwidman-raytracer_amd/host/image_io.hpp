// image_io.hpp — image writers for the host CLI (the display path of the
// reference, Main.cu:317-366 / 382-399, draws the RGBA8 surface into a GL
// texture with texcoord (0,0) at the bottom-left; files are written top row
// first, so the rows are flipped: buffer row 0 = bottom of the screen).
//
// PNG: 8-bit RGBA, zlib stream of stored (uncompressed) deflate blocks —
// no dependency on zlib, every decoder reads it.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace bwrt {

inline uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    crc = ~crc;
    for (size_t i = 0; i < n; i++) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}

inline void put_be32(std::vector<uint8_t>& out, uint32_t v) {
    out.push_back((uint8_t)(v >> 24));
    out.push_back((uint8_t)(v >> 16));
    out.push_back((uint8_t)(v >> 8));
    out.push_back((uint8_t)v);
}

inline void png_chunk(std::vector<uint8_t>& out, const char type[4], const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, crc32_update(0, out.data() + start, out.size() - start));
}

// rgba: width*height*4 bytes, row 0 = bottom (the renderer's orientation).
inline std::vector<uint8_t> encode_png(int width, int height, const uint8_t* rgba) {
    std::vector<uint8_t> raw;  // filter byte 0 + row, top row first
    raw.reserve((size_t)height * (1 + (size_t)width * 4));
    for (int y = height - 1; y >= 0; y--) {
        raw.push_back(0);
        const uint8_t* row = rgba + (size_t)y * width * 4;
        raw.insert(raw.end(), row, row + (size_t)width * 4);
    }
    std::vector<uint8_t> z = {0x78, 0x01};  // zlib header, no compression
    uint32_t a = 1, b = 0;                  // Adler-32
    for (uint8_t c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)(n & 0xFF));
        z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)(~n & 0xFF));
        z.push_back((uint8_t)((~n >> 8) & 0xFF));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    put_be32(z, (b << 16) | a);

    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width);
    put_be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, no filter, no interlace
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", {});
    return out;
}

inline bool write_png(const std::string& path, int width, int height, const uint8_t* rgba) {
    const std::vector<uint8_t> png = encode_png(width, height, rgba);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    return std::fclose(f) == 0 && ok;
}

// Binary PPM (P6), top row first.
inline bool write_ppm(const std::string& path, int width, int height, const uint8_t* rgba) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%d %d\n255\n", width, height);
    for (int y = height - 1; y >= 0; y--)
        for (int x = 0; x < width; x++) std::fwrite(&rgba[((size_t)y * width + x) * 4], 1, 3, f);
    return std::fclose(f) == 0;
}

}  // namespace bwrt
