"""Per-launch EA-level bytes of the forward seam per access-pattern variant (tools/gpu_seam_traffic.sh).

usage: python tools/seam_traffic_table.py <out dir> <variant>...
Reads per variant the counter passes rd (TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum, TCC_BUBBLE_sum,
TCC_EA0_RDREQ_DRAM_sum), wr (TCC_EA0_WRREQ_sum, TCC_EA0_WRREQ_64B_sum) and the kernel trace (durations).
Read bytes = 128 BUBBLE + 64 (RDREQ - BUBBLE - RDREQ_32B) + 32 RDREQ_32B (the TCC_EA interface
bandwidth expression rocprofv3 lists); write bytes = 64 WRREQ_64B + 32 (WRREQ - WRREQ_64B).
The first launch of each run (cold) is dropped.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def counters(d):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "edge_seam" not in row["Kernel_Name"]:
                    continue
                per[int(row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
    ids = sorted(per)[1:]
    keys = set().union(*(per[i].keys() for i in ids)) if ids else set()
    return {k: sum(per[i].get(k, 0.0) for i in ids) / len(ids) for k in keys}


def durations(d):
    us = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "edge_seam" in row["Kernel_Name"]:
                    us.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3))
    us = [u for _, u in sorted(us)][1:]
    return sum(us) / len(us) if us else float("nan")


def main():
    root, variants = sys.argv[1], sys.argv[2:]
    print(f"{'variant':10s} {'us':>7s} {'read MB':>8s} {'(DRAM req MB@64B)':>18s} {'write MB':>9s} {'total MB':>9s} "
          f"{'128B rd':>8s} {'64B rd':>8s} {'32B rd':>8s}")
    for v in variants:
        rd, wr = counters(os.path.join(root, f"{v}_rd")), counters(os.path.join(root, f"{v}_wr"))
        req, r32, bub = rd.get("TCC_EA0_RDREQ_sum", 0), rd.get("TCC_EA0_RDREQ_32B_sum", 0), rd.get("TCC_BUBBLE_sum", 0)
        rbytes = 128 * bub + 64 * (req - bub - r32) + 32 * r32
        wreq, w64 = wr.get("TCC_EA0_WRREQ_sum", 0), wr.get("TCC_EA0_WRREQ_64B_sum", 0)
        wbytes = 64 * w64 + 32 * (wreq - w64)
        dram = rd.get("TCC_EA0_RDREQ_DRAM_sum", 0) * 64
        print(f"{v:10s} {durations(os.path.join(root, v + '_tr')):7.1f} {rbytes / 1e6:8.1f} {dram / 1e6:18.1f} "
              f"{wbytes / 1e6:9.1f} {(rbytes + wbytes) / 1e6:9.1f} {bub:8.0f} {req - bub - r32:8.0f} {r32:8.0f}")


if __name__ == "__main__":
    main()
