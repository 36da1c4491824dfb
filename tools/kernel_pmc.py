#!/usr/bin/env python3
"""Average of every collected counter per dispatch of the kernels whose name contains PATTERN, over
one or more rocprofv3 --pmc pass directories (pmc_counter_collection.csv), plus derived figures:
  valu_per_wave / mfma_per_wave  SQ_INSTS_VALU / SQ_WAVES, SQ_INSTS_MFMA / SQ_WAVES (instruction counts)
  wait_share / inst_wait_share   SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict_share             SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS cycles)
  hbm_bytes                      2 x FETCH_SIZE(KB) x 1024 + WRITE_SIZE(KB) x 1024 (gfx950 FETCH_SIZE is 1/2)
usage: tools/kernel_pmc.py PATTERN DIR [DIR ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(dict)
            for r in csv.DictReader(open(path)):
                if pat in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            for cs in per.values():
                for c, v in cs.items():
                    acc[c].append(v)
    a = {c: sum(v) / len(v) for c, v in acc.items()}
    w = a.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if c in a:
                a[c.lower().replace("sq_insts_", "") + "_per_wave"] = a[c] / w
    if a.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in a:
                a[c.lower().replace("sq_", "") + "_share"] = a[c] / a["SQ_WAVE_CYCLES"]
    if a.get("SQ_LDS_IDX_ACTIVE"):
        a["lds_conflict_share"] = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"]
    if "FETCH_SIZE" in a or "WRITE_SIZE" in a:
        a["hbm_bytes"] = 2 * a.get("FETCH_SIZE", 0.0) * 1024 + a.get("WRITE_SIZE", 0.0) * 1024
    print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in sorted(a.items())}, indent=1))


if __name__ == "__main__":
    main()
