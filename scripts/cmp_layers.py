"""Compare per-layer reports of two measurement dirs (bench.py --layer-report):
dense-conv-path fraction, step rate and the per-layer times that moved.

  python scripts/cmp_layers.py gpurun_out/A gpurun_out/B [batch] [min_delta_us]
"""
import json
import sys


def load(d, b):
    line = json.loads(open(f"{d}/b{b}.json").readline())
    rows = json.load(open(f"{d}/b{b}.layers_per_layer.json"))
    return line, {(r["layer"], r["phase"]): r for r in rows}


def main():
    a, b = sys.argv[1], sys.argv[2]
    bs = [int(sys.argv[3])] if len(sys.argv) > 3 else [16, 32]
    thr = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
    for bt in bs:
        la, ra = load(a, bt)
        lb, rb = load(b, bt)
        da, db = la["roofline"][f"dense_conv_path_b{bt}"], lb["roofline"][f"dense_conv_path_b{bt}"]
        print(f"B{bt}: {la['value']} -> {lb['value']} img/s; dense path {da['frac']} -> {db['frac']} "
              f"({da['kernel_ms_per_step']} -> {db['kernel_ms_per_step']} ms, {da['bytes_per_step_gb']} -> "
              f"{db['bytes_per_step_gb']} GB)")
        ta = sum(r["us"] for r in ra.values())
        tb = sum(r["us"] for r in rb.values())
        print(f"  sum of isolated launches {ta / 1e3:.3f} -> {tb / 1e3:.3f} ms")
        for k in sorted(set(ra) | set(rb)):
            x, y = ra.get(k), rb.get(k)
            ux, uy = (x["us"] if x else 0.0), (y["us"] if y else 0.0)
            if abs(ux - uy) >= thr:
                kx = x["kernel"] if x else "-"
                ky = y["kernel"] if y else "-"
                print(f"  {k[0]:22s} {k[1]:7s} {ux:8.1f} -> {uy:8.1f}  {kx} -> {ky}" if kx != ky else
                      f"  {k[0]:22s} {k[1]:7s} {ux:8.1f} -> {uy:8.1f}  {kx}")


if __name__ == "__main__":
    main()
