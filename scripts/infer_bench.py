"""bench.py's sampler leg alone (improved_sampling 1 x 256^2 fp32/bf16, direct_sampling
64 x 512^2 bf16, SIDD metrics):  python scripts/infer_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import bench
    print(json.dumps(bench.inference_bench(torch.device("cuda", 0))))
