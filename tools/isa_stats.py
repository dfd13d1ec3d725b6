"""Instruction mix of the kernels in a hipcc --save-temps gfx950 .s file (CPU; no GPU needed).

usage: python tools/isa_stats.py file.s [substring ...]
Per kernel whose mangled name contains every substring: instruction count, MFMA, VALU, LDS
(ds_read / ds_write / ds_bpermute / ds_swizzle), DPP, permlane, global / buffer memory, scratch
(spills), s_waitcnt, basic blocks, and the .vgpr_count / .vgpr_spill_count of its metadata."""
import re
import sys


def kernels(s):
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name, start = m.group(1), m.end()
        end = s.find(".Lfunc_end", start)
        yield name, s[start:end]


def main():
    s = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    meta = {}
    for m in re.finditer(r"\.name:\s+(_Z\w+)", s):
        blk = s[max(0, m.start() - 3000):m.start() + 3000]
        v = re.search(r"\.vgpr_count:\s+(\d+)", s[m.start():m.start() + 3000])
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", s[m.start():m.start() + 3000])
        meta[m.group(1)] = (v.group(1) if v else "?", sp.group(1) if sp else "?")
    for name, body in kernels(s):
        if not all(x in name for x in subs):
            continue
        lines = [ln.strip() for ln in body.split("\n") if ln.strip() and not ln.strip().startswith((";", "."))]
        ins = [ln for ln in lines if re.match(r"[a-z_0-9]+", ln) and not ln.endswith(":")]
        c = lambda pat: sum(1 for ln in ins if re.search(pat, ln))  # noqa: E731
        print(name[:110])
        print(f"  insts {len(ins)}  mfma {c(r'^v_mfma')}  valu {c(r'^v_') - c(r'^v_mfma')}  "
              f"ds_read {c(r'^ds_read')}  ds_write {c(r'^ds_write')}  bpermute {c(r'^ds_bpermute')}  "
              f"swizzle {c(r'^ds_swizzle')}  dpp {c(r'row_|quad_perm|row_mirror|row_half')}  permlane {c(r'permlane')}  "
              f"global {c(r'^global_')}  buffer {c(r'^buffer_')}  scratch {c(r'^scratch_')}  waitcnt {c(r'^s_waitcnt')}  "
              f"blocks {sum(1 for ln in lines if ln.endswith(':'))}  vgpr/spill {meta.get(name, ('?', '?'))}")


if __name__ == "__main__":
    main()
