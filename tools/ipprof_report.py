"""Resolve a tools/ipprof.c sample histogram ("offset count" lines, offsets into libm2dec_amd.so) into
the hottest functions (innermost inlined frame) and source lines.
Usage: python3 tools/ipprof_report.py samples.txt [lib.so] [top]"""
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    path = sys.argv[1]
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so")
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    hist = {}
    for line in open(path):
        p = line.split()
        if len(p) == 2:
            hist[int(p[0], 16)] = int(p[1])
    offs = sorted(hist)
    total = sum(hist.values())
    # addr2line -i prints (function, file:line) pairs, innermost first, a variable number per address;
    # -a prints each address first, which marks the boundaries
    out = subprocess.run(["addr2line", "-f", "-i", "-a", "-e", lib] + ["%x" % o for o in offs], capture_output=True,
                         text=True).stdout.splitlines()
    by_fn = collections.Counter()
    by_outer = collections.Counter()
    by_line = collections.Counter()
    i = 0
    k = -1
    frames = []

    def flush():
        if k >= 0 and frames:
            c = hist[offs[k]]
            by_fn[frames[0][0]] += c
            by_outer[frames[-1][0]] += c
            by_line[frames[0][0] + " " + os.path.basename(frames[0][1])] += c

    while i < len(out):
        l = out[i]
        if l.startswith("0x"):
            flush()
            k += 1
            frames = []
            i += 1
            continue
        fn, loc = l, out[i + 1] if i + 1 < len(out) else "?"
        frames.append((fn, loc))
        i += 2
    flush()
    print("samples %d" % total)
    print("-- innermost function")
    for fn, c in by_fn.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, fn))
    print("-- outermost (not inlined) function")
    for fn, c in by_outer.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, fn))
    print("-- source lines")
    for ln, c in by_line.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, ln))


if __name__ == "__main__":
    main()
