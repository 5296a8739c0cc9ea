"""Average PMC counters per kernel over the passes written by scripts/pmc.sh.
FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B: MI355X_MICROARCH.md
HBM section); FETCH_SIZE/WRITE_SIZE are reported in KB per dispatch.

  python scripts/pmc_summary.py [gpurun_out/pmc] [kernel-substring]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name) if "<" not in name else name
    m = re.match(r"(?:void )?(?:[\w:]*::)?(\w+)<(.*)>\(", name)
    if m:
        args = m.group(2).replace("__hip_bfloat16", "bf16").replace("DF16b", "bf16")
        return f"{m.group(1)}<{args}>"
    return name[:60]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if sub and sub not in k:
                continue
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] in ("SQ_WAVE_CYCLES", "FETCH_SIZE", "WRITE_SIZE"):
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    for k, cs in acc.items():
        if sub == "" and not any(s in k for s in ("rdn", "conv", "wgrad", "prelu", "pack", "adam")):
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        out = [f"{k}  n={len(next(iter(cs.values())))}  dur~{sum(dur[k]) / max(1, len(dur[k])):.1f}us"]
        if "FETCH_SIZE" in avg:
            out.append(f"  FETCH x2 = {2 * avg['FETCH_SIZE'] / 1e3:.1f} MB")
        if "WRITE_SIZE" in avg:
            out.append(f"  WRITE = {avg['WRITE_SIZE'] / 1e3:.1f} MB")
        if "TCC_HIT_sum" in avg:
            h, m = avg["TCC_HIT_sum"], avg.get("TCC_MISS_sum", 0)
            out.append(f"  L2 hit = {h / max(1, h + m):.3f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    out.append(f"  {c}/WAVE = {avg[c] / wc:.3f}")
        if "TCP_TCC_READ_REQ_sum" in avg and avg["TCP_TCC_READ_REQ_sum"]:
            out.append(f"  L1->L2 read latency = {avg['TCP_TCC_READ_REQ_LATENCY_sum'] / avg['TCP_TCC_READ_REQ_sum']:.0f} cyc")
        # MFMA pipe utilisation over the dispatch (1024 SIMDs; GRBM_GUI_ACTIVE sums the
        # 8 XCDs' cycles: /8 = the dispatch's cycles, MI355X_MICROARCH.md DVFS note)
        gui = avg.get("GRBM_GUI_ACTIVE")
        if gui:
            cyc = gui / 8.0
            d_us = sum(dur[k]) / max(1, len(dur[k]))
            out.append(f"  clock ~ {cyc / d_us / 1e3:.2f} GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                out.append(f"  MFMA busy = {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f} of the SIMD cycles")
            if "SQ_INSTS_MFMA" in avg:
                out.append(f"  MFMA issue (x16 cyc, 16x16x32) = {16 * avg['SQ_INSTS_MFMA'] / (1024 * cyc):.3f}")
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"  LDS bank-conflict cycles / LDS cycles = "
                       f"{avg.get('SQ_LDS_BANK_CONFLICT', 0) / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
        waves = avg.get("SQ_WAVES") or None
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INST_LEVEL_VMEM", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS",
                  "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",
                  "GRBM_GUI_ACTIVE"):
            if c in avg:
                out.append(f"  {c} = {avg[c]:.4g}")
        print("\n".join(out))


if __name__ == "__main__":
    main()
