#!/usr/bin/env python3
"""Per-plan-entry summary of the SQ counter pass of tools/pmc_session.sh (pass 4).

Prints, per plan entry: waves, MFMA wave-instructions, VALU wave-instructions, LDS bank-conflict
cycles and the MFMA-busy share of the kernel's busy cycles:
  mfma_busy = SQ_INSTS_MFMA x 16 cycles (v_mfma_f32_16x16x32_bf16, one SIMD) / (SQ_BUSY_CYCLES x 4 SIMDs x CUs)
where SQ_BUSY_CYCLES is per SE-aggregated busy clock (rocprofv3 sums it over the 32 SEs, i.e.
8 CUs each).  It is an estimate of MFMA-pipe occupancy during the launch, not a roofline.

usage: tools/pmc_sq.py PASS_DIR/pmc_counter_collection.csv PLAN_NAMES.json
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, names_file = sys.argv[1], sys.argv[2]
    names = json.load(open(names_file))
    rows = list(csv.DictReader(open(path)))
    by_disp = defaultdict(dict)
    kname = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        by_disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        kname[d] = r["Kernel_Name"]
    disps = sorted(by_disp)
    starts = [i for i, d in enumerate(disps) if "patch_im2col" in kname[d]]
    acc = defaultdict(lambda: defaultdict(list))
    for st in starts:
        seq = disps[st:st + len(names)]
        if len(seq) < len(names):
            break
        for nm, d in zip(names, seq):
            for c, v in by_disp[d].items():
                acc[nm][c].append(v)
    # valu_inst = SQ_INSTS_VALU (wave-instructions; SQ_ACTIVE_INST_VALU counts quad-cycles and is only
    # the fallback for round-1 captures)
    print("%-22s %8s %10s %10s %10s %9s" % ("entry", "waves", "mfma_inst", "valu_inst", "lds_confl", "mfma_busy"))
    for nm in dict.fromkeys(names):
        a = {c: sum(v) / len(v) for c, v in acc[nm].items()}
        busy = a.get("SQ_BUSY_CYCLES", 0.0)
        mb = a.get("SQ_INSTS_MFMA", 0.0) * 16 / (busy * 4 * 8) if busy else 0.0
        print("%-22s %8.0f %10.0f %10.0f %10.0f %8.1f%%" % (nm, a.get("SQ_WAVES", 0), a.get("SQ_INSTS_MFMA", 0),
                                                         a.get("SQ_INSTS_VALU", a.get("SQ_ACTIVE_INST_VALU", 0)),
                                                         a.get("SQ_LDS_BANK_CONFLICT", 0), 100 * mb))


if __name__ == "__main__":
    main()
