"""One line per kernel (the N largest by summed dispatch time) from the PMC passes of
scripts/pmc.sh: duration, MFMA busy / issue, LDS bank-conflict cycles per LDS cycle,
LDS-instruction waits, VALU per MFMA, HBM-side bytes (FETCH_SIZE x 2, gfx950:
MI355X_MICROARCH.md), L2 hit rate.

  python scripts/pmc_table.py [gpurun_out/pmc] [N]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?(\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2).replace(' ', '')}>"
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I(.*)", name)
    if m:
        args = re.findall(r"Li(\d+)E|Lb(\d)E|IDF16bE|DF16b", m.group(2))
        vals = [a or ("true" if b == "1" else "false") if (a or b) else "bf16" for a, b in args]
        return f"{m.group(1)}<{','.join(vals)}>"
    return name[:50]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] in ("SQ_WAVE_CYCLES", "FETCH_SIZE", "WRITE_SIZE"):
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    rows = []
    for k, cs in acc.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        d = sum(dur[k]) / max(1, len(dur[k]))
        n = len(cs.get("SQ_WAVE_CYCLES", cs.get("FETCH_SIZE", [0])))
        rows.append((n * d, k, d, a))
    rows.sort(reverse=True)
    hdr = (f"{'kernel':44s} {'us':>6s} {'MFMAbusy':>8s} {'LDSconf':>7s} {'LDSwait':>7s} {'VALU/MFMA':>9s} "
           f"{'FETCHx2MB':>9s} {'WRITEMB':>7s} {'L2hit':>5s} {'GHz':>4s}")
    print(hdr)
    for _, k, d, a in rows[:top]:
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8.0
        busy = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc) if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a else float("nan")
        conf = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"] if a.get("SQ_LDS_IDX_ACTIVE") else float("nan")
        lw = a["SQ_WAIT_INST_LDS"] / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_LDS" in a else float("nan")
        vm = (a["SQ_INSTS_VALU"] - a["SQ_INSTS_MFMA"]) / a["SQ_INSTS_MFMA"] if a.get("SQ_INSTS_MFMA") else float("nan")
        fe = 2 * a.get("FETCH_SIZE", float("nan")) / 1e3
        wr = a.get("WRITE_SIZE", float("nan")) / 1e3
        h, m = a.get("TCC_HIT_sum", 0), a.get("TCC_MISS_sum", 0)
        ghz = cyc / d / 1e3 if cyc and d else float("nan")
        print(f"{k[:44]:44s} {d:6.1f} {busy:8.3f} {conf:7.3f} {lw:7.3f} {vm:9.2f} {fe:9.1f} {wr:7.1f} "
              f"{h / max(1, h + m):5.2f} {ghz:4.2f}")


if __name__ == "__main__":
    main()
