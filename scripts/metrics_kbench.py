"""Device time of rdn_image_metrics (bench.py metrics_bench: 64 SIDD-sized 3 x 256^2
block pairs, a hipGraph of 20 calls) for the in-tree library and, given RDN_LIB,
another build:  python scripts/metrics_kbench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import bench
    r = bench.metrics_bench(torch.device("cuda", 0))
    r["lib"] = os.environ.get("RDN_LIB", "tree")
    print(json.dumps(r))
