"""bench.py's config-1 leg alone: RDUNet(64) on 1 x 3 x 64^2, CPU oracle vs GPU (eager
and ForwardGraph), and the RDUNet(128) 1 x 3 x 256^2 forward:
    python scripts/config1_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import bench
    dev = torch.device("cuda", 0)
    print(json.dumps({"config1_rdunet64_forward": bench.config1_forward(dev),
                      "rdunet128_forward_256": bench.rdunet128_forward(dev)}))
