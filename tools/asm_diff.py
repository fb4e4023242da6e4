#!/usr/bin/env python3
"""Compare the kernels of two `make asm` outputs instruction by instruction
(labels renumbered, comments and directives dropped), so a source change
that should leave a product kernel's ISA unchanged can be checked.

  python tools/asm_diff.py OLD.s NEW.s [--map 'Lb1ELb0E=Lb1ELi0E' ...] [--scratch]

--map OLD=NEW rewrites mangled-name fragments of OLD's symbols (a template
parameter changed type); --scratch lists each kernel's scratch instructions.
"""
import argparse
import re
import sys


def kernels(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end\d+:", text, re.S | re.M):
        lines = []
        for ln in m.group(2).splitlines():
            ln = ln.split(";")[0].strip()
            if not ln or ln.startswith("."):
                continue
            lines.append(re.sub(r"\.LBB\d+_\d+", "L", ln))
        out[m.group(1)] = lines
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    ap.add_argument("--map", action="append", default=[])
    ap.add_argument("--scratch", action="store_true")
    a = ap.parse_args()
    old, new = kernels(a.old), kernels(a.new)
    maps = [m.split("=", 1) for m in a.map]
    same = differ = missing = 0
    for k, body in old.items():
        k2 = k
        for x, y in maps:
            k2 = k2.replace(x, y)
        if k2 not in new:
            missing += 1
            print(f"missing in new: {k2}")
            continue
        if new[k2] == body:
            same += 1
        else:
            differ += 1
            print(f"differs: {k2} ({len(body)} -> {len(new[k2])} instructions)")
    print(f"{same} identical, {differ} differ, {missing} missing; {len(set(new) - set(old))} new-only symbols")
    if a.scratch:
        for k, body in new.items():
            sc = [ln for ln in body if "scratch_" in ln or "buffer_store" in ln or "buffer_load" in ln]
            if sc:
                print(k, len(sc), sc[:6])
    return 1 if differ else 0


if __name__ == "__main__":
    sys.exit(main())
