"""Per-kernel mean of SQ counters from a rocprofv3 --pmc csv directory (tools/pmc_sq.sh).

Columns: launches, mean SQ_WAVE_CYCLES per wave split into WAIT_ANY (parked on s_waitcnt /
barrier), WAIT_INST_ANY (issue stalls, incl. MFMA dependencies and LDS issue), ACTIVE_INST_ANY,
and MFMA busy cycles per SIMD-cycle (quad-cycle units as rocprofv3 reports them).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = re.sub(r"\(.*", "", row["Kernel_Name"].replace("(anonymous namespace)::", ""))[:60]
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, c in sorted(vals.items()):
        mean = {n: sum(v) / len(v) for n, v in c.items()}
        wc = mean.get("SQ_WAVE_CYCLES", 0) or 1
        w = mean.get("SQ_WAVES", 1) or 1
        print(f"{k:60s} n={len(c.get('SQ_WAVES', []))} waves={w:.0f} cyc/wave={wc / w:.0f} "
              f"wait={mean.get('SQ_WAIT_ANY', 0) / wc:.2f} stall={mean.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
              f"(lds {mean.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}) active={mean.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
              f"busy={mean.get('SQ_BUSY_CYCLES', 0):.0f} mfma_busy={mean.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.0f}")


if __name__ == "__main__":
    main()
