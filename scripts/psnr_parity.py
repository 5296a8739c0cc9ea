"""PSNR@sigma=25 parity protocol (last row).

The reference publishes no sigma=25 PSNR and ships no data or checkpoints, so
parity is shown by training twice from the same state and comparing the
denoising quality reached:

* identical initial weights (``oracle.weights.make_params``, counter hash),
* identical seeded synthetic data: smooth procedural RGB textures quantised to
  uint8, Gaussian sigma=25 noise added in uint8 space and clipped exactly as
  ``dataset_creation/custom_dataset.py:83-87``, then ToTensor + Normalize(0.5, 0.5)
  -> [-1, 1] (``data_loader.py:35-38``),
* identical timestep draws t ~ U{0..T} (``diffusion_RDUnet.py:87``),
* the same step: interpolation, UNet, Charbonnier, backward, clip 1.0
  (``diffusion_RDUnet.py:76-115``) followed by ``torch.optim.Adam`` every step.

Leg A is this build on the GPU (``train_step_device`` through librdunet_hip, fp32
mode; optionally bf16).  Leg B is the CPU oracle (``oracle/rdunet_ref.py``, the
reference's aten math in fp32 NCHW).  Both then denoise a held-out set with
``improved_sampling`` (T=20: 40 UNet forwards, ``diffusion_RDUnet.py:38-50``) and
PSNR is computed per image with the ``hyperparams_search.py:11-28`` convention
(denormalise to [0, 1], 20*log10(1/RMSE), mean over images).  Target:
|PSNR_gpu - PSNR_cpu| <= 0.05 dB.

Paired design (``--seeds N``): every seed is one pair (same init, data, t draws
for both legs); the statistic is the per-seed difference d_i = PSNR_gpu,i -
PSNR_cpu,i, reported with its mean, standard deviation and a two-sided 95 %
Student-t confidence interval.  Training is chaotic (rounding differences of a
few ulps grow over the steps: the oracle against itself from 1e-6-perturbed
weights differs by up to 0.2 dB per seed), so the interval, not one seed, is the
evidence; it is narrower than +-0.05 dB at N ~ 12.  Each seed also checks the
inference path alone: the GPU-trained weights denoise the held-out set on the
GPU and in the oracle, d_inf = PSNR difference at identical weights.

  python scripts/psnr_parity.py [--steps 150] [--bf16] [--out profiles/x.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def textures(n: int, size: int, seed: int) -> np.ndarray:
    """Smooth procedural RGB images, uint8 [n, size, size, 3]: per channel a few
    low-frequency oriented sinusoids plus Gaussian blobs."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(size, dtype=np.float64) / size, np.arange(size, dtype=np.float64) / size,
                         indexing="ij")
    out = np.empty((n, size, size, 3), np.uint8)
    for i in range(n):
        img = np.zeros((size, size, 3))
        for c in range(3):
            f = np.zeros((size, size))
            for _ in range(4):
                fx, fy = rng.uniform(-4, 4, 2)
                f += rng.uniform(0.3, 1.0) * np.sin(2 * np.pi * (fx * xx + fy * yy) + rng.uniform(0, 2 * np.pi))
            for _ in range(3):
                cx, cy, s = rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(0.05, 0.25)
                f += rng.uniform(-1.5, 1.5) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
            img[..., c] = f
        lo, hi = img.min(), img.max()
        img = (img - lo) / max(hi - lo, 1e-9)
        out[i] = np.round(16 + 223 * img).astype(np.uint8)
    return out


def noisy_pairs(clean_u8: np.ndarray, sigma: float, seed: int):
    """custom_dataset.py:84-86 noise (float32 += N(0, sigma) float64 -> clip -> uint8),
    then ToTensor + Normalize(0.5, 0.5): (noisy, clean) float32 NCHW in [-1, 1]."""
    rng = np.random.default_rng(seed)
    noisy = clean_u8.astype(np.float32)
    noisy += rng.normal(scale=sigma, size=clean_u8.shape)
    noisy = np.clip(noisy, 0, 255).astype(np.uint8)

    def norm(a):
        return ((a.transpose(0, 3, 1, 2).astype(np.float32) / np.float32(255)) - np.float32(0.5)) / np.float32(0.5)

    return torch.from_numpy(np.ascontiguousarray(norm(noisy))), torch.from_numpy(np.ascontiguousarray(norm(clean_u8)))


def psnr_per_image(den: torch.Tensor, clean: torch.Tensor) -> float:
    """hyperparams_search.py:11-16,24-28: denormalise, per-image 20*log10(1/RMSE), mean."""
    d, c = den.double() * 0.5 + 0.5, clean.double() * 0.5 + 0.5
    vals = [20 * math.log10(1.0 / math.sqrt(torch.mean((d[i] - c[i]) ** 2).item())) for i in range(d.size(0))]
    return float(np.mean(vals))


def make_data(args):
    tr_u8 = textures(args.n_train, args.size, args.seed)
    ev_u8 = textures(args.n_eval, args.size, args.seed + 1)
    tr_noisy, tr_clean = noisy_pairs(tr_u8, args.sigma, args.seed + 2)
    ev_noisy, ev_clean = noisy_pairs(ev_u8, args.sigma, args.seed + 3)
    rng = np.random.default_rng(args.seed + 4)
    sched = []
    for _ in range(args.steps):
        idx = rng.choice(args.n_train, args.batch, replace=False)
        t = rng.integers(0, args.timesteps + 1, args.batch)   # U{0..T}, diffusion_RDUnet.py:87
        sched.append((torch.from_numpy(idx), torch.from_numpy(t)))
    return tr_noisy, tr_clean, ev_noisy, ev_clean, sched


def run_gpu(args, params, data, dtype):
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
    tr_noisy, tr_clean, ev_noisy, ev_clean, sched = data
    dev = torch.device("cuda")
    unet = vm.RDUNet_T(base_filters=args.base_filters)
    model = DiffusionModel(unet, timesteps=args.timesteps)
    model.load_state_dict({"unet." + k: torch.from_numpy(v) for k, v in params.items()})
    model = model.to(dev)
    unet.set_compute_dtype(dtype)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    trn, trc = tr_noisy.to(dev), tr_clean.to(dev)
    t0 = time.perf_counter()
    losses = []
    for idx, t in sched:
        idx = idx.to(dev)
        loss = train_step_device(model, trc[idx], trn[idx], opt, clip_value=1.0, t=t.to(dev))
        opt.step()
        losses.append(loss)
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    model.eval()
    with torch.no_grad():
        den = torch.cat([model.improved_sampling(ev_noisy[i:i + args.eval_batch].to(dev)).cpu()
                         for i in range(0, ev_noisy.size(0), args.eval_batch)])
    losses = [float(v) for v in torch.stack(losses).detach().cpu()]
    return {"psnr": psnr_per_image(den, ev_clean), "loss_first": losses[0], "loss_last": losses[-1],
            "train_s": round(t_train, 2), "losses": losses,
            "_state": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}}


def oracle_eval_psnr(args, state_dict, data):
    """The oracle's improved_sampling + PSNR with given (GPU-trained) weights."""
    from oracle import rdunet_ref as R
    _, _, ev_noisy, ev_clean, _ = data
    P = {k[5:]: v.detach().cpu().float() for k, v in state_dict.items() if k.startswith("unet.")}

    def fn(x, tt):
        return R.rdunet_t_forward(P, x, tt)

    with torch.no_grad():
        den = torch.cat([R.improved_sampling(fn, ev_noisy[i:i + args.eval_batch], args.timesteps)
                         for i in range(0, ev_noisy.size(0), args.eval_batch)])
    return psnr_per_image(den, ev_clean)


def run_cpu(args, params, data):
    from oracle import rdunet_ref as R
    tr_noisy, tr_clean, ev_noisy, ev_clean, sched = data
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    P = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
    opt = torch.optim.Adam(list(P.values()), lr=args.lr)
    t0 = time.perf_counter()
    losses = []
    for idx, t in sched:
        loss, _, grads, _ = R.train_step(P, tr_clean[idx], tr_noisy[idx], t, args.timesteps, clip_value=1.0)
        for k, p in P.items():
            p.grad = grads[k]
        opt.step()
        losses.append(float(loss))
    t_train = time.perf_counter() - t0

    def fn(x, tt):
        return R.rdunet_t_forward(P, x, tt)

    with torch.no_grad():
        den = torch.cat([R.improved_sampling(fn, ev_noisy[i:i + args.eval_batch], args.timesteps)
                         for i in range(0, ev_noisy.size(0), args.eval_batch)])
    return {"psnr": psnr_per_image(den, ev_clean), "loss_first": losses[0], "loss_last": losses[-1],
            "train_s": round(t_train, 2), "threads": torch.get_num_threads(), "losses": losses}


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--n-train", type=int, default=64)
    ap.add_argument("--n-eval", type=int, default=16)
    ap.add_argument("--eval-batch", type=int, default=16)
    ap.add_argument("--base-filters", type=int, default=32)
    ap.add_argument("--timesteps", type=int, default=20)
    ap.add_argument("--sigma", type=float, default=25.0)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--bf16", action="store_true", help="also train the bf16 build (report only)")
    ap.add_argument("--seeds", type=int, default=1, help="independent repetitions (PSNR averaged)")
    ap.add_argument("--self-noise", action="store_true",
                    help="also train the CPU oracle from ~1e-6-perturbed weights: the protocol's noise floor")
    ap.add_argument("--keep-losses", action="store_true")
    ap.add_argument("--part", choices=("all", "gpu", "cpu"), default="all",
                    help="run only the GPU legs (on the MI355X box) or only the CPU-oracle legs (any host); "
                         "--merge pairs the two files by seed")
    ap.add_argument("--merge", nargs="+", default=None, metavar="JSON",
                    help="combine --part gpu / --part cpu outputs (same config) and report")
    ap.add_argument("--out", default="")
    return ap


def _one(args, seed):
    from oracle import rdunet_ref as R
    from oracle.weights import make_params
    a = argparse.Namespace(**vars(args))
    a.seed = seed
    params = make_params(R.param_shapes(a.base_filters), seed)
    data = make_data(a)
    r = {"seed": seed, "psnr_noisy_input": psnr_per_image(data[2], data[3])}
    gpu, cpu = args.part in ("all", "gpu"), args.part in ("all", "cpu")
    if gpu:
        r["gpu_fp32"] = run_gpu(a, params, data, "fp32")
        print(f"seed {seed}: gpu fp32 psnr {r['gpu_fp32']['psnr']:.4f}", flush=True)
        # inference parity at identical weights: the GPU-trained model, denoised by the oracle
        r["oracle_eval_of_gpu_weights_psnr"] = oracle_eval_psnr(a, r["gpu_fp32"].pop("_state"), data)
        r["delta_inference_db"] = r["gpu_fp32"]["psnr"] - r["oracle_eval_of_gpu_weights_psnr"]
        if args.bf16:
            r["gpu_bf16"] = run_gpu(a, params, data, "bf16")
            r["gpu_bf16"].pop("_state")
    if not cpu:
        return r
    r["cpu_oracle_fp32"] = run_cpu(a, params, data)
    print(f"seed {seed}: cpu fp32 psnr {r['cpu_oracle_fp32']['psnr']:.4f}", flush=True)
    if args.self_noise:
        # the protocol's own noise floor: the same CPU oracle from weights perturbed by
        # ~1e-6 relative (a few fp32 ulps, the size of GPU-vs-CPU rounding differences)
        rng = np.random.default_rng(seed + 7)
        pert = {k: (v * (1 + 1e-6 * rng.standard_normal(v.shape))).astype(np.float32) for k, v in params.items()}
        r["cpu_oracle_fp32_perturbed"] = run_cpu(a, pert, data)
    if not gpu:
        return r
    return _finish(args, r)


def _finish(args, r):
    lg, lc = r["gpu_fp32"]["losses"], r["cpu_oracle_fp32"]["losses"]
    rel = [abs(x - y) / abs(y) for x, y in zip(lg, lc)]
    r["loss_traj_max_rel_diff"] = max(rel)
    r["loss_traj_first_step_over_1e-3"] = next((i for i, v in enumerate(rel) if v > 1e-3), None)
    for leg in ("gpu_fp32", "cpu_oracle_fp32", "cpu_oracle_fp32_perturbed", "gpu_bf16"):
        if leg in r and not args.keep_losses:
            r[leg].pop("losses")
    return r


def paired_stats(d):
    """Mean, sd and two-sided 95 % Student-t interval of per-seed differences."""
    n = len(d)
    out = {"n": n, "per_seed_db": [float(x) for x in d], "mean_db": float(np.mean(d))}
    if n > 1:
        from scipy import stats
        sd = float(np.std(d, ddof=1))
        half = float(stats.t.ppf(0.975, n - 1)) * sd / math.sqrt(n)
        out.update(sd_db=sd, ci95=[out["mean_db"] - half, out["mean_db"] + half], ci95_halfwidth_db=half)
    return out


def run(args):
    seeds = [args.seed + 100 * i for i in range(args.seeds)]
    runs = [_one(args, s) for s in seeds]
    if args.part != "all":
        return {"part": args.part, "config": {k: getattr(args, k) for k in (
                    "steps", "batch", "size", "n_train", "n_eval", "base_filters", "timesteps", "sigma", "lr",
                    "seed", "seeds")}, "runs": runs}
    return summarize(args, runs)


def merge(args):
    """Pair --part gpu and --part cpu outputs by seed (configs must agree)."""
    parts = [json.load(open(f)) for f in args.merge]
    cfg = {k: v for k, v in parts[0]["config"].items() if k not in ("seed", "seeds")}
    by_seed = {}
    for prt in parts:
        if {k: v for k, v in prt["config"].items() if k not in ("seed", "seeds")} != cfg:
            raise SystemExit("configs differ")
        for r in prt["runs"]:
            by_seed.setdefault(r["seed"], {}).update(r)
    runs = [r for _, r in sorted(by_seed.items()) if "gpu_fp32" in r and "cpu_oracle_fp32" in r]
    for k, v in cfg.items():
        setattr(args, k, v)
    args.seed, args.seeds = runs[0]["seed"], len(runs)
    args.self_noise = all("cpu_oracle_fp32_perturbed" in r for r in runs)
    args.bf16 = all("gpu_bf16" in r for r in runs)
    runs = [_finish(args, r) for r in runs]
    return summarize(args, runs)


def summarize(args, runs):
    mean = lambda leg: float(np.mean([r[leg]["psnr"] for r in runs]))
    res = {"protocol": "SURVEY.md §8d PSNR@sigma=25: identical init, data and t draws; Adam every step; "
                       "improved_sampling T=20 on a held-out set; hyperparams_search.py PSNR convention; "
                       "mean over seeds",
           "config": {k: getattr(args, k) for k in ("steps", "batch", "size", "n_train", "n_eval", "base_filters",
                                                    "timesteps", "sigma", "lr", "seed", "seeds")},
           "psnr_noisy_input": float(np.mean([r["psnr_noisy_input"] for r in runs])),
           "psnr_gpu_fp32": mean("gpu_fp32"), "psnr_cpu_oracle_fp32": mean("cpu_oracle_fp32")}
    res["delta_db"] = res["psnr_gpu_fp32"] - res["psnr_cpu_oracle_fp32"]
    d = np.array([r["gpu_fp32"]["psnr"] - r["cpu_oracle_fp32"]["psnr"] for r in runs])
    res["paired"] = paired_stats(d)
    res["pass_0p05db"] = bool(abs(res["delta_db"]) <= 0.05)
    res["ci95_within_0p05db"] = bool(res["paired"]["ci95"][0] >= -0.05 and res["paired"]["ci95"][1] <= 0.05) \
        if len(d) > 1 else None
    di = np.array([r["delta_inference_db"] for r in runs])
    res["inference_parity"] = {"per_seed_db": [float(x) for x in di], "max_abs_db": float(np.max(np.abs(di)))}
    if args.self_noise:
        res["psnr_cpu_oracle_fp32_perturbed"] = mean("cpu_oracle_fp32_perturbed")
        res["self_noise_delta_db"] = res["psnr_cpu_oracle_fp32_perturbed"] - res["psnr_cpu_oracle_fp32"]
    if args.self_noise:
        res["self_noise_paired"] = paired_stats(np.array([r["cpu_oracle_fp32_perturbed"]["psnr"] -
                                                          r["cpu_oracle_fp32"]["psnr"] for r in runs]))
    if args.bf16:
        res["psnr_gpu_bf16"] = mean("gpu_bf16")
        res["delta_bf16_vs_fp32_db"] = res["psnr_gpu_bf16"] - res["psnr_gpu_fp32"]
        res["bf16_vs_oracle_paired"] = paired_stats(np.array([r["gpu_bf16"]["psnr"] - r["cpu_oracle_fp32"]["psnr"]
                                                              for r in runs]))
    res["runs"] = runs
    return res


def main():
    args = parser().parse_args()
    if args.part != "all":
        args.keep_losses = True     # the merge compares the loss trajectories
    res = merge(args) if args.merge else run(args)
    s = json.dumps(res, indent=1)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
