#!/usr/bin/env python
"""Derived metrics from rocprofv3 --pmc passes (profiles/pmc/*_counter_collection.csv): per kernel
and grid shape -- duration, bf16 MFMA TFLOP/s (MOPS x 512), MFMA-busy share of the active CUs'
cycles, LDS bank-conflict cycles per LDS instruction, HBM-side bytes (FETCH_SIZE / WRITE_SIZE,
KiB) and L2 hit rate."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc")
for prog in ("bench", "lin", "mw"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, f"{prog}_p*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
            key = (name, r["Grid_Size"], r["Workgroup_Size"])
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (f, r["Dispatch_Id"])
            disp[key].add(did)
            dur[key][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    print(f"## {prog}")
    print("| kernel | grid | dispatches | time/dispatch us | bf16 TFLOP/s | MFMA busy / (active CUs x cycles) | LDS conflict cycles / LDS inst | HBM read KiB | HBM write KiB | L2 hit % | VALU / MFMA | SALU / MFMA |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for key in sorted(agg, key=lambda k: -sum(dur[k].values())):
        c = agg[key]
        n_pass = len({f for f, _ in disp[key]})
        ndisp = len(disp[key]) / max(1, n_pass)
        t = sum(dur[key].values()) / max(1, len(dur[key]))
        flops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512 / ndisp
        tf = flops / t / 1e12 if t > 0 else 0
        waves = c.get("SQ_WAVES", 0) / ndisp
        wg = int(key[2])
        cus = min(256, max(1, waves * 64 / wg)) if waves else 0
        gui = c.get("GRBM_GUI_ACTIVE", 0) / ndisp / 8      # summed over the 8 XCDs
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / ndisp
        util = 100 * mfma / (gui * cus) if gui and cus else 0
        lds = c.get("SQ_INSTS_LDS", 0)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        l2 = 100 * hit / (hit + miss) if hit + miss else 0
        nm = c.get("SQ_INSTS_MFMA", 0)
        valu = f"{c['SQ_INSTS_VALU'] / nm:.1f}" if nm and "SQ_INSTS_VALU" in c else "-"
        salu = f"{c['SQ_INSTS_SALU'] / nm:.1f}" if nm and "SQ_INSTS_SALU" in c else "-"
        print(f"| {key[0]} | {key[1]} | {ndisp:.0f} | {t * 1e6:.1f} | {tf:.2f} | {util:.1f}% | {conf:.2f} | "
              f"{c.get('FETCH_SIZE', 0) / ndisp:.0f} | {c.get('WRITE_SIZE', 0) / ndisp:.0f} | {l2:.1f} | {valu} | {salu} |")
    print()
