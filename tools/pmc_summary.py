"""Summarise rocprofv3 --pmc CSVs (tools/gpu_round.sh, tools/gpu_pmc.sh): per kernel name, counters averaged per
dispatch (VALU / LDS / stall counters of the query kernels).

  python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "phip::"
    vals = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per_dispatch = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat not in row["Kernel_Name"]:
                    continue
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per_dispatch[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = row["Kernel_Name"]
                meta[row["Kernel_Name"]] = (row["Grid_Size"], row["LDS_Block_Size"], row["VGPR_Count"],
                                            row["SGPR_Count"], row["Scratch_Size"])
        for (d, c), v in per_dispatch.items():
            vals[names[d]][c].append(v)
    for k, cs in vals.items():
        print(k, "grid,lds,vgpr,sgpr,scratch =", meta[k])
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
