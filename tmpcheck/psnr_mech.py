import json, sys, time
sys.path.insert(0, "tests")
import test_gpu_psnr as T
T.FIXTURE = "tmpcheck/psnr_partial.json"
T.MIN_SEEDS = 10
t0 = time.time()
for k in range(T.SHARDS):
    T.test_psnr_sigma25_shard(k)
    print("shard", k, time.time() - t0, flush=True)
try:
    T.test_psnr_sigma25_paired_vs_oracle_fixture()
    print("PASS", time.time() - t0)
except AssertionError as e:
    print("ASSERT", e, time.time() - t0)
