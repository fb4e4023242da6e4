// rt_diag.h — diagnostic hooks of the render kernels (device side).
//
// The product build compiles every hook here to nothing: the hooks are empty
// inline functions or empty macros unless one of the diagnostic defines is
// set (tools/stamps_run.py, tools/phase_lanes.sh, tools/gtimes_run.py and the
// BVH check build pass them).  Keeping them here leaves the kernels' round
// loops reading as the product; `make asm` + tools/asm_diff.py check that
// the product ISA does not change with them.
//
//   RT_STAMPS        per-phase wave-cycle sums and utilisation counters of
//                    the sorted kernel (SortedStamps) and the BVH refill
//                    kernel (RefillStamps) -> K.stamps (BWRT_STAMPS=1);
//   RT_PHASE_TWICE   1 / 2 / 3 / 4: the sorted kernel runs its closest hit /
//                    RANDDIR task / SPEC task / path-end fold a second time on
//                    opaque copies of the inputs (results kept alive, never
//                    used): the PMC deltas against the plain build are that
//                    phase's VALU instructions and lane-cycles;
//   RT_GTIMES        per-group start / end times (100 MHz realtime) ->
//                    K.stamps[2g], [2g+1], and (refill kernel) each lane's
//                    pixel-done time -> K.stamps[2 * 65536 + 64g + lane]
//                    (BWRT_GTIMES=file; buffer RT_GTIMES_WORDS words);
//   RT_BVH_CHECK     the refill kernel re-runs each query through the
//                    brute-force loop and logs disagreements to K.stamps.
#pragma once

#include "rt_layout.h"
#include "rt_path.h"

#ifndef RT_PHASE_TWICE
#define RT_PHASE_TWICE 0
#endif

// ---- opaque copies (RT_PHASE_TWICE): the second run cannot be folded into
// the first, and its results stay live without being used
__device__ __forceinline__ float opq(float x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ f3 opq3(f3 v) { return mk(opq(v.x), opq(v.y), opq(v.z)); }
__device__ __forceinline__ void keep(float x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void keep_i(int x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ Xorwow opq_rs(Xorwow r) {
    Xorwow q;
    q.d = __float_as_uint(opq(__uint_as_float(r.d)));
    q.v0 = __float_as_uint(opq(__uint_as_float(r.v0)));
    q.v1 = __float_as_uint(opq(__uint_as_float(r.v1)));
    q.v2 = __float_as_uint(opq(__uint_as_float(r.v2)));
    q.v3 = __float_as_uint(opq(__uint_as_float(r.v3)));
    q.v4 = __float_as_uint(opq(__uint_as_float(r.v4)));
    return q;
}
// value readers of a fold: the product's (identity) and the opaque one
struct DiagIdent {
    __device__ __forceinline__ float operator()(float v) const { return v; }
};
struct DiagOpaque {
    __device__ __forceinline__ float operator()(float v) const { return opq(v); }
};

// RT_TWICE_*: the phase named by RT_PHASE_TWICE once more, on opaque inputs
#if RT_PHASE_TWICE == 1
#define RT_TWICE_HIT(QUADS, K, o, d)                                    \
    do {                                                                \
        float _t2;                                                      \
        int _id2;                                                       \
        closest_hit_brute<QUADS>(K, opq3(o), opq3(d), _t2, _id2);       \
        keep(_t2);                                                      \
        keep_i(_id2);                                                   \
    } while (0)
#else
#define RT_TWICE_HIT(QUADS, K, o, d) \
    do {                             \
    } while (0)
#endif
#if RT_PHASE_TWICE == 2
#define RT_TWICE_RANDDIR(rs, nrm)                          \
    do {                                                   \
        Xorwow _r2 = opq_rs(rs);                           \
        const f3 _x = random_direction(_r2, opq3(nrm));    \
        keep(_x.x + _x.y + _x.z);                          \
        keep_i((int)_r2.v4);                               \
    } while (0)
#else
#define RT_TWICE_RANDDIR(rs, nrm) \
    do {                          \
    } while (0)
#endif
#if RT_PHASE_TWICE == 3
#define RT_TWICE_SPEC(rs, dd, nrm, h2)                                                                     \
    do {                                                                                                   \
        Xorwow _r2 = opq_rs(rs);                                                                           \
        float _k2;                                                                                         \
        const f3 _x = specular_scatter(_r2, opq3(dd), opq3(nrm), opq((h2).x), opq((h2).z), opq((h2).y), _k2); \
        keep(_x.x + _x.y + _x.z + _k2);                                                                    \
        keep_i((int)_r2.v4);                                                                               \
    } while (0)
#else
#define RT_TWICE_SPEC(rs, dd, nrm, h2) \
    do {                               \
    } while (0)
#endif
// fold_path(reader, lx, ly, lz): the kernel's path-end fold with its loads
// passed through `reader`
#if RT_PHASE_TWICE == 4
#define RT_TWICE_FOLD(K, fold_path)                                         \
    do {                                                                    \
        float _mx = opq((K).bg[0]), _my = opq((K).bg[1]), _mz = opq((K).bg[2]); \
        fold_path(DiagOpaque(), _mx, _my, _mz);                             \
        keep(_mx + _my + _mz);                                              \
    } while (0)
#else
#define RT_TWICE_FOLD(K, fold_path) \
    do {                            \
    } while (0)
#endif

// ---- RT_GTIMES: group and lane times
__device__ __forceinline__ void diag_group_start(const rt_kparams& K) {
#ifdef RT_GTIMES
    if (threadIdx.x == 0 && K.stamps && 2 * (unsigned long long)blockIdx.x + 1 < RT_GTIMES_WORDS)
        K.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
}
// (multi-wave groups: after a barrier, so the time is the group's last wave)
template <bool SYNC>
__device__ __forceinline__ void diag_group_end(const rt_kparams& K) {
#ifdef RT_GTIMES
    if (SYNC) __syncthreads();
    if (threadIdx.x == 0 && K.stamps && 2 * (unsigned long long)blockIdx.x + 1 < RT_GTIMES_WORDS)
        K.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}
// a lane's pixels are done (the first call per lane counts; 64-lane groups)
struct LaneDone {
#ifdef RT_GTIMES
    bool done = false;
    __device__ __forceinline__ void mark(const rt_kparams& K) {
        const unsigned long long i = 2ull * 65536 + 64ull * blockIdx.x + threadIdx.x;
        if (!done && K.stamps && i < RT_GTIMES_WORDS) K.stamps[i] = __builtin_amdgcn_s_memrealtime();
        done = true;
    }
#else
    __device__ __forceinline__ void mark(const rt_kparams&) {}
#endif
};

// ---- RT_BVH_CHECK: the brute-force loop on the refill kernel's finished
// query; a disagreement is logged to K.stamps: [0] count, then 16 words per
// record
__device__ __forceinline__ void diag_bvh_check(const rt_kparams& K, f3 o, f3 d, float best_t, int best_id, int depth) {
#ifdef RT_BVH_CHECK
    float bt;
    int bi;
    closest_hit_brute(K, o, d, bt, bi);
    if ((bi != best_id || (bi >= 0 && bt != best_t && !(bt != bt && best_t != best_t))) && K.stamps) {
        const unsigned long long k = atomicAdd(&K.stamps[0], 1ull);
        if (k < 4096) {
            unsigned long long* rec = K.stamps + 16 + 16 * k;
            rec[0] = __float_as_uint(o.x);
            rec[1] = __float_as_uint(o.y);
            rec[2] = __float_as_uint(o.z);
            rec[3] = __float_as_uint(d.x);
            rec[4] = __float_as_uint(d.y);
            rec[5] = __float_as_uint(d.z);
            rec[6] = __float_as_uint(best_t);
            rec[7] = (unsigned)best_id;
            rec[8] = __float_as_uint(bt);
            rec[9] = (unsigned)bi;
            rec[10] = (unsigned)depth;
        }
    }
#else
    (void)K, (void)o, (void)d, (void)best_t, (void)best_id, (void)depth;
#endif
}

// ---- RT_STAMPS: the sorted kernel's wave-cycle split.  stamp(k) adds the
// cycles since the previous stamp to phase k: [7] round top, [0] first
// barrier, [1] posting, [2] second barrier, [3] execute, [4] third barrier,
// [5] take-back, [6] I-phase; utilisation counters (lane 0 of each wave
// adds): [0] rounds, [1] front waves, [2] front tasks, [3] rejection-loop
// wave trips, [4] rejection lane trips, [5] spec waves, [6] spec tasks,
// [7] I-phase waves, [8] I-phase rays -> K.stamps[8 + i]
struct SortedStamps {
#ifdef RT_STAMPS
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long u[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long prev;
    int rej = 0;
    __device__ __forceinline__ SortedStamps() : prev(__builtin_amdgcn_s_memtime()) {}
    __device__ __forceinline__ void stamp(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[k] += t - prev;
        prev = t;
    }
    __device__ __forceinline__ int* rej_ptr() { return &rej; }
    static __device__ __forceinline__ int wave_max(int v) {
        for (int m = 1; m < 64; m <<= 1) v = max(v, __shfl_xor(v, m));
        return v;
    }
    static __device__ __forceinline__ int wave_sum(int v) {
        for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
        return v;
    }
    __device__ __forceinline__ void exec(bool do_front, bool do_spec) {
        const int itl = (do_front && !do_spec) ? rej : 0;
        rej = 0;
        const unsigned long long bf = __ballot(do_front), bs = __ballot(do_spec);
        const int mx = wave_max(itl), sm = wave_sum(itl);
        if ((threadIdx.x & 63) == 0) {
            u[0] += 1;
            u[1] += bf != 0;
            u[2] += __popcll(bf);
            u[3] += mx;
            u[4] += sm;
            u[5] += bs != 0;
            u[6] += __popcll(bs);
        }
    }
    __device__ __forceinline__ void rays(bool has_ray) {
        const unsigned long long br = __ballot(has_ray);
        if ((threadIdx.x & 63) == 0) {
            u[7] += br != 0;
            u[8] += __popcll(br);
        }
    }
    __device__ __forceinline__ void flush(const rt_kparams& K) {
        if ((threadIdx.x & 63) == 0 && K.stamps) {
            for (int k = 0; k < 8; k++) atomicAdd(&K.stamps[k], acc[k]);
            for (int k = 0; k < 9; k++) atomicAdd(&K.stamps[8 + k], u[k]);
        }
    }
#else
    __device__ __forceinline__ void stamp(int) {}
    __device__ __forceinline__ int* rej_ptr() { return nullptr; }
    __device__ __forceinline__ void exec(bool, bool) {}
    __device__ __forceinline__ void rays(bool) {}
    __device__ __forceinline__ void flush(const rt_kparams&) {}
#endif
};

// the BVH refill kernel's: cycles in [0] refill / shading, [1] node steps,
// [2] leaf tests; counts [3] refill passes, [4] node-loop iterations, [5]
// leaf batches -> K.stamps[0..5]
struct RefillStamps {
#ifdef RT_STAMPS
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long prev;
    __device__ __forceinline__ RefillStamps() : prev(__builtin_amdgcn_s_memtime()) {}
    __device__ __forceinline__ void stamp(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[k] += t - prev;
        prev = t;
    }
    __device__ __forceinline__ void count(int k) { acc[k] += 1; }
    __device__ __forceinline__ void flush(const rt_kparams& K) {
        if ((threadIdx.x & 63) == 0 && K.stamps)
            for (int k = 0; k < 6; k++) atomicAdd(&K.stamps[k], acc[k]);
    }
#else
    __device__ __forceinline__ void stamp(int) {}
    __device__ __forceinline__ void count(int) {}
    __device__ __forceinline__ void flush(const rt_kparams&) {}
#endif
};
