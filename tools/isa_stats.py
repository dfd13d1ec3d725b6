"""Per-kernel ISA statistics of a hipcc -S output: loads, vmcnt(0) waits, branches.

usage: python tools/isa_stats.py <file.s>
A kernel whose vector loads are each followed by `s_waitcnt vmcnt(0)` (or branched around)
runs its memory accesses one at a time.
"""
import re
import sys


def main():
    text = open(sys.argv[1]).read().splitlines()
    cur, stats = None, {}
    for line in text:
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            stats[cur] = {"global_load": 0, "buffer_load": 0, "vmcnt0": 0, "vmcnt": 0, "cbranch": 0, "lines": 0}
            continue
        if cur is None:
            continue
        s = stats[cur]
        s["lines"] += 1
        if "global_load" in line:
            s["global_load"] += 1
        if "buffer_load" in line:
            s["buffer_load"] += 1
        if "s_waitcnt" in line and "vmcnt(0)" in line:
            s["vmcnt0"] += 1
        elif "s_waitcnt" in line and "vmcnt(" in line:
            s["vmcnt"] += 1
        if "s_cbranch" in line:
            s["cbranch"] += 1
        if "s_endpgm" in line:
            cur = None
    for k, s in stats.items():
        name = re.sub(r"^_ZN5gasfm(12_GLOBAL__N_1)?\d+", "", k)[:60]
        print(f"{name:60s} " + " ".join(f"{a}={b}" for a, b in s.items()))


if __name__ == "__main__":
    main()
