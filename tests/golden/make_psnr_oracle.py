"""Fixture generator for tests/test_gpu_psnr.py: the CPU-oracle leg of the
PSNR@sigma=25 paired experiment (scripts/psnr_parity.py protocol),
precomputed here because 144 seeds x 120 oracle train steps take ~1 h of host CPU.

Per seed (oracle/rdunet_ref.py, the reference's aten math in fp32 NCHW, ONE thread
so the trajectory is reproducible): identical init (oracle.weights.make_params),
identical procedural sigma=25 data and t draws (psnr_parity.make_data), 120 steps of
train_step (diffusion_RDUnet.py:76-115) + torch.optim.Adam(lr 2e-4), then the
oracle's own improved_sampling (T=20, diffusion_RDUnet.py:38-50) on the 16 held-out
64x64 images and on one held-out 256x256 image (the same fully convolutional
weights), PSNR per hyperparams_search.py:11-16,24-28.

  python tests/golden/make_psnr_oracle.py --workers 6 --out tests/golden/psnr_sigma25_oracle.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

CFG = dict(steps=120, batch=8, size=64, n_train=64, n_eval=16, eval_batch=16, base_filters=32, timesteps=20,
           sigma=25.0, lr=2e-4)
SEED0, SEED_STRIDE = 4000, 37


def eval_256(seed, sigma=25.0):
    """The 256x256 held-out image of a seed: (noisy, clean) [1, 3, 256, 256]."""
    import psnr_parity as PP
    return PP.noisy_pairs(PP.textures(1, 256, seed + 5), sigma, seed + 6)


def one_seed(seed):
    import torch
    torch.set_num_threads(1)
    import psnr_parity as PP
    from oracle import rdunet_ref as R
    from oracle.weights import make_params
    a = argparse.Namespace(**CFG, seed=seed)
    params = make_params(R.param_shapes(a.base_filters), seed)
    data = PP.make_data(a)
    tr_noisy, tr_clean, ev_noisy, ev_clean, sched = data
    P = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
    opt = torch.optim.Adam(list(P.values()), lr=a.lr)
    losses = []
    for idx, t in sched:
        loss, _, grads, _ = R.train_step(P, tr_clean[idx], tr_noisy[idx], t, a.timesteps, clip_value=1.0)
        for k, p in P.items():
            p.grad = grads[k]
        opt.step()
        losses.append(float(loss))

    def fn(x, tt):
        return R.rdunet_t_forward(P, x, tt)

    with torch.no_grad():
        den = R.improved_sampling(fn, ev_noisy, a.timesteps)
        n256, c256 = eval_256(seed, a.sigma)
        den256 = R.improved_sampling(fn, n256, a.timesteps)
    return {"seed": seed, "noisy": PP.psnr_per_image(ev_noisy, ev_clean), "oracle": PP.psnr_per_image(den, ev_clean),
            "noisy_256": PP.psnr_per_image(n256, c256), "oracle_256": PP.psnr_per_image(den256, c256),
            "loss_first": losses[0], "loss_last": losses[-1]}


def main():
    import concurrent.futures as cf
    import multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=144)
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                  "psnr_sigma25_oracle.json"))
    args = ap.parse_args()
    seeds = [SEED0 + SEED_STRIDE * i for i in range(args.seeds)]
    done = {}
    if os.path.exists(args.out):      # resume
        for r in json.load(open(args.out))["runs"]:
            done[r["seed"]] = r
    todo = [s for s in seeds if s not in done]
    t0 = time.time()

    def save():
        runs = [done[s] for s in seeds if s in done]
        with open(args.out + ".tmp", "w") as f:   # (atomic: the run may be stopped at any time)
            json.dump({"config": CFG, "seed0": SEED0, "seed_stride": SEED_STRIDE, "threads_per_seed": 1,
                       "generator": "tests/golden/make_psnr_oracle.py", "runs": runs}, f, indent=0)
        os.replace(args.out + ".tmp", args.out)

    with cf.ProcessPoolExecutor(args.workers, mp_context=mp.get_context("spawn")) as ex:
        futs = {ex.submit(one_seed, s): s for s in todo}
        for f in cf.as_completed(futs):
            r = f.result()
            done[r["seed"]] = r
            save()
            print(f"[{time.time() - t0:7.0f}s] seed {r['seed']}: noisy {r['noisy']:.3f} oracle {r['oracle']:.3f} "
                  f"256: {r['noisy_256']:.3f} -> {r['oracle_256']:.3f} ({len(done)}/{len(seeds)})", flush=True)
    save()


if __name__ == "__main__":
    main()
