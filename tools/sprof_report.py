#!/usr/bin/env python3
"""Flat and inclusive profile from tools/sprof.c's SPROF_RAW samples, symbolised with
addr2line (function names incl. static ones; -i: the innermost inlined function counts
as the frame).  Development tool.

    python tools/sprof_report.py raw.txt [--top 60] [--incl] [--callers]
"""
import collections
import subprocess
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 60
    samples = [ln.split() for ln in open(path)]
    addrs = collections.defaultdict(set)
    for fr in samples:
        for f in fr:
            if ":" in f:
                mod, off = f.rsplit(":", 1)
                addrs[mod].add(off)
    name = {}
    for mod, offs in addrs.items():
        offs = sorted(offs)
        r = subprocess.run(["addr2line", "-f", "-C", "-e", mod] + ["0x" + o for o in offs],
                           capture_output=True, text=True)
        lines = r.stdout.splitlines()
        for i, o in enumerate(offs):
            fn = lines[2 * i] if 2 * i < len(lines) else "?"
            if fn == "??":
                fn = f"[{mod.rsplit('/', 1)[-1]}]"
            name[(mod, o)] = fn[:150]
    self_c, incl_c = collections.Counter(), collections.Counter()
    for fr in samples:
        seen = set()
        for d, f in enumerate(fr):
            if ":" not in f:
                continue
            mod, off = f.rsplit(":", 1)
            fn = name[(mod, off)]
            if d == 0:
                self_c[fn] += 1
            if fn not in seen:
                incl_c[fn] += 1
                seen.add(fn)
    n = len(samples)
    print(f"# {n} samples")
    if "--callers" in sys.argv:                 # first frame in the main binary below a libc frame
        callers = collections.Counter()
        for fr in samples:
            if not fr or ":" not in fr[0] or "libc" not in fr[0]:
                continue
            for f in fr[1:]:
                if ":" in f and "libc" not in f and "libstdc++" not in f:
                    fn = name[tuple(f.rsplit(":", 1))]
                    if fn.startswith(("std::", "__gnu_cxx::", "void std::", "decltype", "operator new")):
                        continue                 # allocator/container plumbing: keep walking
                    callers[fn] += 1
                    break
        for fn, c in callers.most_common(top):
            print(f"{100 * c / n:6.2f} {fn}")
        return
    if "--lines" in sys.argv:                   # self samples by source line (build with -g)
        lines_c = collections.Counter()
        for mod in addrs:
            pass
        firsts = collections.defaultdict(list)
        for fr in samples:
            if fr and ":" in fr[0]:
                mod, off = fr[0].rsplit(":", 1)
                firsts[mod].append(off)
        for mod, offs in firsts.items():
            uniq = sorted(set(offs))
            r = subprocess.run(["addr2line", "-i", "-C", "-e", mod] + ["0x" + o for o in uniq],
                               capture_output=True, text=True)
            # with -i an address may print several lines (inline chain): keep the first
            out, k = {}, 0
            outl = r.stdout.splitlines()
            r2 = subprocess.run(["addr2line", "-C", "-e", mod] + ["0x" + o for o in uniq], capture_output=True, text=True)
            for o, ln in zip(uniq, r2.stdout.splitlines()):
                out[o] = ln.rsplit("/", 1)[-1]
            for o in offs:
                lines_c[out.get(o, "?")] += 1
        for ln, c in lines_c.most_common(top):
            print(f"{100 * c / n:6.2f} {ln}")
        return
    key = incl_c if "--incl" in sys.argv else self_c
    for fn, c in key.most_common(top):
        print(f"{100 * self_c[fn] / n:6.2f} {100 * incl_c[fn] / n:6.2f} {fn}")


if __name__ == "__main__":
    main()
