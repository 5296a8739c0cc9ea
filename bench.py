"""Throughput bench: the RDUNet_T diffusion TRAIN STEP (BASELINE.json metric,
config 2 at N=1: batch 16 per GPU, 256x256x3 synthetic sigma in {15,25,50},
bf16 compute with fp32 master weights/accumulation).

One step = t draw + interpolation + RDUNet_T(32) forward + Charbonnier loss +
backward + global-norm clip (1.0) + fused AdamW update (lr 1e-4, wd 1e-4),
i.e. train_step_checkpointed followed by optimizer.step() EVERY step (the
reference steps every 4th batch; stepping every batch is strictly more work).
For N>1 (torchrun, one process per GPU) each rank trains on its own 16 images
and gradients are all-reduced over RCCL, bucketed and overlapped with the
backward (weak scaling).

Prints ONE JSON line (rank 0).  Extra objects:
  roofline      dominant kernel instantiation, achieved algorithmic TFLOP/s or
                GB/s measured with HIP events on the compute stream over the timed
                region, against the MI355X peak (MI355X_MICROARCH.md)
                `traffic`: HBM bytes per launch of that kernel from rocprofv3 PMC
                counters (FETCH_SIZE x2 + WRITE_SIZE, separate passes of a short
                child run of this bench; MI355X_MICROARCH.md HBM section)
  cpu_baseline  the CPU oracle (torch fp32 NCHW, the reference's aten math) train
                step at batch 2 on this host's cores, bounded sample
  inference     the samplers on the same GPU: improved_sampling latency on one
                256x256 image (the reference publishes ~1.29 s) and config 4's
                direct_sampling at batch 64 x 512x512
Progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # dense MFMA (MI355X_MICROARCH.md chip table)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
MEASURED_HBM_GBS = 6290.0   # float4 copy on MI355X (MI355X_MICROARCH.md chip table)


class EventTracer:
    """engine.TRACER: HIP events around the launches of selected kernels."""

    def __init__(self, keys=None):
        self.keys = keys      # None = every traced launch
        self.records = []     # (info, start, end)

    def start(self, info, stream=None):
        """Events go on the stream the traced kernel is launched on (the
        engine's weight-gradient side stream for wgrad launches)."""
        if self.keys is not None and info[2] not in self.keys:
            return None
        s = torch.cuda.Event(enable_timing=True)
        s.record(stream)
        return (info, s, stream)

    def stop(self, tok):
        e = torch.cuda.Event(enable_timing=True)
        e.record(tok[2])
        self.records.append((tok[0], tok[1], e))

    def per_layer(self):
        torch.cuda.synchronize()
        rows = {}
        for info, s, e in self.records:
            k = (info[1], info[0])
            r = rows.setdefault(k, {"ms": 0.0, "n": 0, "flops": info[3], "bytes": info[4], "kernel": info[2]})
            r["ms"] += s.elapsed_time(e)
            r["n"] += 1
        return [{"layer": k[0], "phase": k[1], "kernel": v["kernel"], "us": round(1e3 * v["ms"] / v["n"], 2),
                 "tflops": round(v["flops"] / (v["ms"] / v["n"] * 1e-3) / 1e12, 1),
                 "gbs": round(v["bytes"] / (v["ms"] / v["n"] * 1e-3) / 1e9, 1)} for k, v in rows.items()]

    def summary(self):
        torch.cuda.synchronize()
        by = {}
        for info, s, e in self.records:
            ms = s.elapsed_time(e)
            k = info[2]
            d = by.setdefault(k, {"ms": 0.0, "n": 0, "flops": 0.0, "bytes": 0.0, "phases": set()})
            d["ms"] += ms
            d["n"] += 1
            d["flops"] += info[3]
            d["bytes"] += info[4]
            d["phases"].add(info[0])
        return by


def extra_configs(dev, args):
    """The same train step at north_star's batch 32 (bf16, with the residual-dense
    conv path's HBM roofline from a serialised profiling pass) and at the
    reference's own precision (fp32, batch 16).  Rank 0 of a 1-GPU run only."""
    out = {}
    for key, batch, dtype, warm, steps in (("b32", 32, "bf16", 3, args.steps), ("fp32", 16, "fp32", 2, max(20, args.steps))):
        _log(f"extra config {key}: batch {batch} {dtype}")
        tr = Trainer(dev, batch, args.size, args.base_filters, dtype, graph=args.graph == "on")
        for i in range(warm):
            tr.step(i)
        profs = [tr.profile() for _ in range(PROFILE_PASSES)] if key == "b32" else None
        if profs is not None:   # replays again before the timed steps (the serialised eager passes
            for i in range(warm):   # left the clocks low: two B32 lines read 1852 / 1912 against 2022-2062)
                tr.step(i)
        el, loss = tr.timed(steps)
        r = {"per_gpu_batch": batch, "dtype": dtype, "steps": steps, "graph": args.graph == "on",
             "ms_per_step": round(el * 1e3 / steps, 3),
             "images_per_s": round(batch * steps / el, 2), "final_loss": round(loss.item(), 5)}
        if profs is not None:
            r["dense_conv_path"] = dense_conv_path_median(profs, batch)
        out[key] = r
        del tr, profs
        torch.cuda.empty_cache()
    return out


def cpu_baseline(seconds=12.0, batch=16, size=256, steps=3):
    """The CPU oracle's train step (fp32, torch aten on the host cores), at the
    headline's per-GPU batch: one batch-2 warm-up step, then `steps` whole batch
    steps (at least 3), the MEDIAN step time reported (`seconds` is kept for the
    command line; a B16 step takes ~12 s on 16 host cores)."""
    from oracle import rdunet_ref as R
    from oracle.weights import make_params
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(threads)
    params = {k: torch.from_numpy(v) for k, v in make_params(R.param_shapes(32), 0).items()}
    g = torch.Generator().manual_seed(0)
    clean = torch.rand(batch, 3, size, size, generator=g) * 2 - 1
    noisy = clean + (25 / 255 * 2) * torch.randn(batch, 3, size, size, generator=g)
    t = torch.randint(0, 21, (batch,), generator=g)
    R.train_step(params, clean[:2], noisy[:2], t[:2], 20)  # warm-up (allocator, threads)
    ts = []
    for _ in range(max(3, steps)):
        t0 = time.perf_counter()
        R.train_step(params, clean, noisy, t, 20)
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    # BASELINE.md "What is timed" legs 2-3: the reference's own batch-2 step (SURVEY §6's
    # 2.02 img/s on 8 vCPU) and its published inference timing, improved_sampling
    # (T = 20: 40 UNet forwards) on one 256x256 image (evaluate_model.py:126-133)
    t2 = []
    for _ in range(3):
        t0 = time.perf_counter()
        R.train_step(params, clean[:2], noisy[:2], t[:2], 20)
        t2.append(time.perf_counter() - t0)
    med2 = sorted(t2)[1]
    x1 = noisy[:1]
    with torch.no_grad():
        t0 = time.perf_counter()
        R.improved_sampling(lambda xx, tt: R.rdunet_t_forward(params, xx, tt), x1, 20)
        t_samp = time.perf_counter() - t0
    return {"value": round(batch / med, 4), "unit": "images/s", "cores": torch.get_num_threads(),
            "kind": "port", "step_s_median": round(med, 3), "step_s_all": [round(x, 3) for x in ts],
            "train_step_b2": {"images_per_s": round(2 / med2, 4), "step_s_median": round(med2, 3),
                              "step_s_all": [round(x, 3) for x in t2]},
            "improved_sampling_256_b1_s": round(t_samp, 3),
            "sample": f"median of {len(ts)} oracle train steps (fwd+Charbonnier+bwd+clip) of RDUNet_T(32) fp32 at "
                      f"batch {batch} x 3x{size}x{size} on the host CPU ({sum(ts):.1f}s timed); also the batch-2 "
                      f"step (median of 3) and one improved_sampling call (T=20) on 1x3x{size}x{size}"}


def config1_forward(dev, reps=5):
    """BASELINE config 1: RDUNet (UNet/RDUNet_model.py:117-186, base_filters 64)
    forward on one 1x3x64x64 Gaussian-noise tensor.  The reference runs it on the
    CPU (the oracle restates that path, timed here on the host cores: median of
    `reps`); the same call through this build on the GPU (fp32, parity mode) is
    timed beside it and compared (rel-L2)."""
    from oracle import rdunet_ref as R
    from oracle.weights import make_params
    import vub_image_denoising_amd as vm
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(threads)
    params = {k: torch.from_numpy(v) for k, v in make_params(R.param_shapes(64, 3, 3), 2).items()}
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        R.rdunet_forward(params, x)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            y_cpu = R.rdunet_forward(params, x)
            ts.append(time.perf_counter() - t0)
    from vub_image_denoising_amd.sampling import ForwardGraph
    m = vm.RDUNet(channels=3, base_filters=64)
    m.load_state_dict(params)
    m = m.to(dev).eval()
    xg = x.to(dev)
    with torch.no_grad():
        m(xg)
        torch.cuda.synchronize()
        tg = []
        for _ in range(20):
            t0 = time.perf_counter()
            y = m(xg)
            torch.cuda.synchronize()
            tg.append(time.perf_counter() - t0)
        fg = ForwardGraph(m, tuple(xg.shape))
        yg = fg(xg).clone()
        torch.cuda.synchronize()
        tgr = []
        for _ in range(20):
            t0 = time.perf_counter()
            fg(xg)
            torch.cuda.synchronize()
            tgr.append(time.perf_counter() - t0)
    rel = ((y.cpu().double() - y_cpu.double()).norm() / y_cpu.double().norm()).item()
    return {"workload": "RDUNet(channels=3, base_filters=64) forward, 1x3x64x64 Gaussian noise",
            "cpu_ms_median": round(1e3 * sorted(ts)[reps // 2], 3), "cpu_cores": torch.get_num_threads(),
            "gpu_fp32_ms_median": round(1e3 * sorted(tg)[10], 3),
            "gpu_fp32_graph_ms_median": round(1e3 * sorted(tgr)[10], 3),
            "graph_equals_eager": bool(torch.equal(yg, y)),
            "gpu_vs_cpu_rel_l2": float(f"{rel:.3e}"),
            "note": "host wall per call (eager: ~70 launches issued from Python; graph: one hipGraph replay)"}


def rdunet128_forward(dev, reps=20):
    """The plain RDUNet(base_filters=128) -- the reference's module-level baseline
    model (UNet/RDUNet_model.py:189) -- on one 3x256x256 image, the shape of its
    published ~0.01 s single-forward inference time (evaluate_Unet_diffusion/
    evaluate_model.py:126-143 timing): hipGraph-captured forward,
    fp32 (the reference's precision) and bf16, with TF/s and the fraction of peak."""
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.sampling import ForwardGraph
    torch.manual_seed(11)
    m = vm.RDUNet(channels=3, base_filters=128).to(dev).eval()
    x = torch.rand(1, 3, 256, 256, device=dev) * 2 - 1
    res = {"workload": "RDUNet(channels=3, base_filters=128) forward, 1x3x256x256", "published_s": 0.01}
    for dt in ("fp32", "bf16"):
        m.set_compute_dtype(dt)
        fg = ForwardGraph(m, tuple(x.shape))
        fg(x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fg(x)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        eng = m._rdn_engines[(1, 256, 256, torch.float32 if dt == "fp32" else torch.bfloat16, False)][0]
        flops = sum(L.extra["info"]["fwd"][3] for L in eng.layers)
        peak = PEAK_F32_TFLOPS if dt == "fp32" else PEAK_BF16_TFLOPS
        res[dt] = {"ms": round(ms, 4), "tflops": round(flops / (ms * 1e-3) / 1e12, 1),
                   "frac_of_peak": round(flops / (ms * 1e-3) / 1e12 / peak, 4),
                   "speedup_vs_published": round(10.0 / ms, 1)}
        del fg
    res["gflop"] = round(flops / 1e9, 2)
    del m
    torch.cuda.empty_cache()
    return res


def _log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _kernel_sig(name):
    """(base name, integer template args, gate flag) of a kernel instantiation, from
    the launch probe's key ('conv3_halo_kernel<bf16,64,2,64,gate>') or from a
    rocprofv3 kernel name (Itanium-mangled or demangled).  Element types are
    dropped (one bench run uses one dtype)."""
    import re
    if name.startswith("_Z"):
        end = name.find("_kernelI")
        if end < 0:
            return None
        end += len("_kernel")
        base = None
        for start in range(end - 1, 0, -1):     # <length><identifier> ending at `end`
            n = str(end - start)
            if name[start - len(n):start] == n and (name[start].isalpha() or name[start] == "_"):
                base = name[start:end]
                break
        if base is None:
            return None
        rest, ints, gate = name[end + 1:], [], False
        while rest and rest[0] != "E":
            t = re.match(r"DF16b|f|Li(\d+)E|Lb([01])E", rest)
            if not t:
                return None
            if t.group(1) is not None:
                ints.append(int(t.group(1)))
            elif t.group(2) is not None:
                gate = t.group(2) == "1"
            rest = rest[t.end():]
        return base, ints, gate
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    if not m:
        return None
    ints, gate = [], False
    for tok in (x.strip() for x in m.group(2).split(",")):
        if tok.isdigit():
            ints.append(int(tok))
        elif tok in ("gate", "true"):
            gate = True
    return m.group(1), ints, gate


def pmc_traffic(key, args, timeout=240):
    """HBM bytes per launch of kernel `key`, from rocprofv3 PMC counters collected
    in two child runs of this bench (MI355X_MICROARCH.md, HBM section: FETCH_SIZE and
    WRITE_SIZE in separate --pmc passes beside --kernel-trace only; on gfx950
    FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled).  Returns
    (bytes or None, note)."""
    import csv
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not on PATH"
    want = _kernel_sig(key)
    kb = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="rdn_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["rocprofv3", "--kernel-trace", "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--no-cpu-baseline", "--steps", "2",
               "--warmup", "1", "--batch", str(args.batch), "--size", str(args.size), "--base-filters",
               str(args.base_filters), "--dtype", args.dtype]
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            shutil.rmtree(d, ignore_errors=True)
            return None, f"{ctr} pass timed out"
        vals = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") == ctr and _kernel_sig(row.get("Kernel_Name", "")) == want:
                        vals.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if rc != 0 or not vals:
            return None, f"{ctr} pass rc={rc}, {len(vals)} matching dispatches"
        kb[ctr] = sum(vals) / len(vals)
    return (2.0 * kb["FETCH_SIZE"] + kb["WRITE_SIZE"]) * 1024.0, "rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE, KiB"


def inference_bench(dev, base_filters=32):
    """The sampler paths on the same GPU (hipGraph-captured, SamplerGraph):
    improved_sampling (2T = 40 UNet forwards, diffusion_RDUnet.py:38-50) on one
    256x256 image — the reference's published ≈1.29 s/image — and
    config 4's direct_sampling at batch 64 x 512x512."""
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel
    from vub_image_denoising_amd.sampling import SamplerGraph
    torch.manual_seed(7)
    dm = DiffusionModel(vm.RDUNet_T(base_filters=base_filters), timesteps=20).to(dev).eval()
    res = {}

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    x1 = torch.rand(1, 3, 256, 256, device=dev) * 2 - 1
    for dt in ("fp32", "bf16"):
        dm.unet.set_compute_dtype(dt)
        g = SamplerGraph(dm, tuple(x1.shape))
        res[f"improved_sampling_256_b1_{dt}_ms"] = round(1e3 * timed(lambda: g(x1), 5), 3)
        del g
    res["published_improved_sampling_256_b1_s"] = 1.29
    res["speedup_vs_published_fp32"] = round(1.29e3 / res["improved_sampling_256_b1_fp32_ms"], 1)
    dm.unet.set_compute_dtype("bf16")
    x64 = torch.rand(64, 3, 512, 512, device=dev) * 2 - 1
    g = SamplerGraph(dm, tuple(x64.shape), direct=True)
    t = timed(lambda: g(x64), 3)
    # (forward-only batches past 2^23 pixels run in image chunks, engine.run_unet: the
    # engines are keyed by the chunk's batch)
    eng = next(p[0] for k, p in dm.unet._rdn_engines.items() if k[1:] == (512, 512, torch.bfloat16, False))
    flops = sum(L.extra["info"]["fwd"][3] for L in eng.layers) * 64 / eng.B
    res["direct_sampling_512_b64_bf16"] = {"ms_per_call": round(1e3 * t, 2), "images_per_s": round(64 / t, 1),
                                           "tflops": round(flops / t / 1e12, 1),
                                           "frac_of_peak": round(flops / t / 1e12 / PEAK_BF16_TFLOPS, 4),
                                           "engine_batch": eng.B}
    del g, x64
    dm.unet._rdn_engines.clear()
    torch.cuda.empty_cache()
    res["sidd_metrics"] = metrics_bench(dev)
    return res


def metrics_bench(dev, n=64, size=256):
    """SIDD evaluation metrics (rdn_image_metrics: PSNR + SSIM, evaluate_SIDD.py:63-64)
    on a batch of n 3 x size x size block pairs resident in HBM; HBM-bound, the
    algorithmic bytes are the two fp32 images read once."""
    from vub_image_denoising_amd.metrics import image_metrics
    g = torch.Generator(device=dev).manual_seed(5)
    a = torch.rand(n, 3, size, size, generator=g, device=dev) * 2 - 1
    b = (a + 0.1 * torch.randn(n, 3, size, size, generator=g, device=dev)).clamp_(-1, 1)
    reps = 20
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        torch.cuda.synchronize()
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    def eager():
        for _ in range(reps):
            image_metrics(a, b, 2.0)

    eager()
    host_ms = timed(eager)
    # the device time of a call: `reps` calls captured in one hipGraph (the eager loop
    # above is bound by the ~3 torch allocations + launch per call, not by the kernel)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        eager()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        eager()
    graph.replay()
    ms = timed(graph.replay)
    nbytes = 2 * a.numel() * 4
    return {"blocks": n, "block": [3, size, size], "ms_per_batch": round(ms, 4), "eager_ms_per_call": round(host_ms, 4),
            "blocks_per_s": round(n / (ms * 1e-3), 1), "achieved_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "peak_GBs": PEAK_HBM_GBS, "frac": round(nbytes / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "timing": "hipGraph of 20 calls (both kernels), inputs resident in HBM",
            "note": "per-block skimage on the host (reference) is not timed here"}


class GraphCaptureError(RuntimeError):
    """The hipGraph capture of a data-parallel step raised; `trainer` is usable eagerly."""

    def __init__(self, trainer):
        super().__init__("graph capture of the data-parallel train step failed")
        self.trainer = trainer


class Trainer:
    """One RDUNet_T train step (the timed unit) for a (per-GPU batch, dtype):
    synthetic seeded data resident in HBM, FusedAdamW every step."""

    def __init__(self, dev, batch, size, base_filters, dtype, rank=0, world=1, graph=False):
        import vub_image_denoising_amd as vm
        from vub_image_denoising_amd.ddp import GradSync
        from vub_image_denoising_amd.diffusion_RDUnet import DiffusionModel, train_step_device
        from vub_image_denoising_amd.optim import FusedAdamW
        self.batch = batch
        torch.manual_seed(1234)
        self.unet = vm.RDUNet_T(base_filters=base_filters).to(dev).set_compute_dtype(dtype)
        self.model = DiffusionModel(self.unet, timesteps=20)
        # synthetic data resident in HBM: one batch per sigma, rank-specific seed
        gen = torch.Generator(device=dev).manual_seed(1234 + 7919 * rank)
        self.batches = []
        for sigma in (15.0, 25.0, 50.0):
            clean = torch.rand(batch, 3, size, size, generator=gen, device=dev) * 2 - 1
            noisy = clean + (sigma / 255.0 * 2.0) * torch.randn(batch, 3, size, size, generator=gen, device=dev)
            self.batches.append((noisy, clean))
        torch.manual_seed(99 + rank)  # t draws (torch.randint on the device)
        self._train_step = train_step_device
        self.opt = None
        self.graph = None
        self.step(0)  # builds the flat parameter buffer and the engine
        self.opt = FusedAdamW(self.model.parameters(), lr=1e-4, weight_decay=1e-4)
        if world > 1:
            self.unet._rdn_flat.grad_sync = GradSync(self.unet._rdn_flat, bucket_mb=25.0)
            if graph:   # device-clock stamps around the all-reduce tail, replayed with the graph
                self.unet._rdn_flat.grad_sync.stamps = torch.zeros(3, dtype=torch.int64, device=dev)
        self.graph = None
        if graph:   # the whole step as one hipGraph replay (train_graph.TrainStepGraph)
            from vub_image_denoising_amd.train_graph import TrainStepGraph
            try:
                self.graph = TrainStepGraph(self.model, self.opt, tuple(self.batches[0][0].shape), 'uniform', 1.0)
            except Exception as e:
                if world == 1:
                    raise
                self.graph = None
                raise GraphCaptureError(self) from e

    def step(self, i):
        noisy, clean = self.batches[i % 3]
        if self.graph is not None and not self.eager:
            return self.graph(clean, noisy)
        opt = self.opt if self.opt is not None else self
        loss = self._train_step(self.model, clean, noisy, opt, "uniform", 1.0)
        if self.opt is not None:
            self.opt.step()
        return loss

    eager = False   # profiling passes run the step eagerly (per-launch events)

    def zero_grad(self, set_to_none=True):   # stands in for the optimizer on the first step
        for p in self.model.parameters():
            p.grad = None

    def profile(self):
        """One step with every conv launch timed alone (backward serialised)."""
        from vub_image_denoising_amd import engine as E
        prof = EventTracer()
        E.TRACER, E.SERIAL_BWD = prof, True
        self.eager = True
        try:
            self.step(0)
        finally:
            E.TRACER, E.SERIAL_BWD = None, False
            self.eager = False
        return prof

    def timed(self, steps, world=1, tracer=None):
        from vub_image_denoising_amd import engine as E
        E.TRACER = tracer
        self.eager = tracer is not None
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            loss = self.step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        E.TRACER = None
        self.eager = False
        return el, loss

    def host_issue_ms(self, n=10):
        """Host time to issue one step (median; the GPU drained before each)."""
        ts = []
        for i in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.step(i)
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        return round(1e3 * sorted(ts)[n // 2], 3)


DENSE_LEVELS = (0, 1)
PROFILE_PASSES = 3   # serialised profiling passes behind each dense_conv_path figure (median reported)


def dense_conv_path_median(profs, batch):
    """dense_conv_path of each profiling pass; the median pass reported, with the
    spread of the passes (verdict r04: one pass per line was not reproducible)."""
    rs = sorted((dense_conv_path(p, batch) for p in profs), key=lambda r: r["frac"])
    med = dict(rs[len(rs) // 2])
    med["passes"] = len(rs)
    med["frac_min"], med["frac_max"] = rs[0]["frac"], rs[-1]["frac"]
    med["frac_all"] = [r["frac"] for r in rs]
    return med


def dense_conv_path(prof, batch):
    """HBM roofline of north_star's "residual-dense conv path": the 3x3 convs of the
    level-0/1 DenoisingBlocks (Unet_model.py:72-89; block_0_* / block_1_* conv_0..3)
    in forward, input gradient and weight gradient.  achieved = their algorithmic
    bytes (each operand read once, each output written once, engine._build_info) /
    their summed isolated kernel time of one step."""
    import re
    byts, bmin, ms, n = 0.0, 0.0, 0.0, 0
    for info, s, e in prof.records:
        m = re.match(r"block_(\d)_\d\.conv_[\d-]+$", info[1])   # (conv_0-2: the fused level-0 launch)
        if m and int(m.group(1)) in DENSE_LEVELS and info[0] != "prelu":   # (convs only)
            byts += info[4]
            bmin += info[5] if len(info) > 5 else info[4]
            ms += s.elapsed_time(e)
            n += 1
    gbs = byts / (ms * 1e-3) / 1e9
    gmin = bmin / (ms * 1e-3) / 1e9
    return {"batch": batch, "levels": list(DENSE_LEVELS), "launches": n, "bytes_per_step_gb": round(byts / 1e9, 3),
            "kernel_ms_per_step": round(ms, 3), "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "frac_of_measured_copy_bw": round(gbs / MEASURED_HBM_GBS, 4),
            "frac_dense3_fused_minimal": round(gmin / PEAK_HBM_GBS, 4),
            "bytes_per_step_gb_dense3_fused_minimal": round(bmin / 1e9, 3),
            "note": "isolated (serialised-backward) launch times; bytes incl. the fused PReLU-backward gate reads; "
                    "frac counts the fused level-0 conv_0..2 launch at the three convs' bytes (SURVEY §8d per-conv "
                    "definition), frac_dense3_fused_minimal at its own minimal bytes (x read once)"}


# a rank whose hipGraph capture of the data-parallel step raised exits with this code;
# the launcher then starts the whole job again, eagerly (--graph off), in fresh processes
EXIT_GRAPH_FAILED = 3


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# a rank that outlives the deadline (every rank hung in a collective, say) is killed
# and the job exits with this code, so a caller's clock never runs out on a silent run
EXIT_DEADLINE = 124


def deadline_s(args):
    """Wall-clock budget of one rank / one launch: `--deadline-s`, else a bound
    derived from the work (start-up, capture and profiling passes, the B32 / fp32
    lines and CPU legs of a 1-GPU run, 4 s per timed or warm-up step)."""
    if args.deadline_s and args.deadline_s > 0:
        return float(args.deadline_s)
    return 900.0 + 4.0 * (args.steps + args.warmup)


def _run_ranks(n, argv, grace_s=60.0, deadline=None):
    """Start n ranks of this bench (fresh child processes, one per GPU: RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on
    127.0.0.1) and wait for them.  When a rank fails the others get `grace_s` to
    finish before their process groups are killed (a rank left waiting in a
    collective would never return); past `deadline` seconds every rank still
    running is killed and reported as EXIT_DEADLINE.  Returns the ranks' exit codes."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RDN_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      start_new_session=True))

    def kill_running():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

    failed_at = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            return rcs
        if deadline is not None and time.monotonic() - t0 > deadline:
            hung = [r for r, rc in enumerate(rcs) if rc is None]
            _log(f"deadline of {deadline:.0f} s passed with rank(s) {hung} still running: killing them")
            kill_running()
            rcs = [p.wait() for p in procs]
            return [EXIT_DEADLINE if r in hung else rc for r, rc in enumerate(rcs)]
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            kill_running()
            return [p.wait() for p in procs]
        time.sleep(0.2)


def start_watchdog(seconds, rank):
    """Per-rank deadline under ANY launcher (torchrun included): a daemon thread
    ends the process with EXIT_DEADLINE if it is still running after `seconds`
    (a rank stuck inside a collective never returns to Python to notice)."""
    import threading

    def fire():
        print(f"bench.py rank {rank}: deadline of {seconds:.0f} s passed, exiting with {EXIT_DEADLINE}",
              file=sys.stderr, flush=True)
        os._exit(EXIT_DEADLINE)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def launch(args, argv):
    """`--gpus N` (N > 1) without a launcher's environment: run the N ranks as child
    processes of this one -- which never touches the GPU itself -- so that
    `python bench.py --gpus N` measures N GPUs exactly as
    `torchrun --nproc-per-node N bench.py --gpus N` does.  If a rank reports that
    the hipGraph capture of the RCCL step raised (exit EXIT_GRAPH_FAILED), the job
    runs again from fresh processes with --graph off."""
    dl = deadline_s(args)
    rcs = _run_ranks(args.gpus, argv, deadline=dl)
    if EXIT_GRAPH_FAILED in rcs and args.graph == "on":
        _log(f"graph capture or first replay failed on a rank (exit codes {rcs}); running the job again eagerly "
             f"(--graph off)")
        rcs = _run_ranks(args.gpus, [*argv, "--graph", "off"], deadline=dl)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--base-filters", type=int, default=32)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--layer-report", default="", help="write a per-kernel time table (json) here")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes (roofline.traffic)")
    ap.add_argument("--no-inference", action="store_true", help="skip the sampler measurements")
    ap.add_argument("--no-extra", action="store_true", help="skip the batch-32 and fp32 train-step lines")
    ap.add_argument("--graph", choices=["on", "off"], default="on",
                    help="time the step as one hipGraph replay (train_graph.TrainStepGraph) or eagerly")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="ranks report RANK/LOCAL_RANK/WORLD_SIZE as JSON and exit before touching the GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only for eager plumbing tests)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (plumbing tests of N > 1 on a 1-GPU box; gloo, --graph off)")
    ap.add_argument("--deadline-s", type=float, default=0.0,
                    help="wall-clock limit per rank and per launch (0: derived from --steps / --warmup)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run as "
              f"{args.gpus} GPUs", file=sys.stderr)
        sys.exit(2)
    if world > 1 or args.deadline_s:
        # (under bench.py's own launcher its deadline fires first; under torchrun this is the only one)
        start_watchdog(deadline_s(args) + (30.0 if os.environ.get("RDN_BENCH_LAUNCHED") else 0.0), rank)
    if args.launch_dry_run:
        if os.environ.get("RDN_BENCH_DRY_GRAPH_FAIL") and args.graph == "on":   # tests of the eager restart
            sys.exit(EXIT_GRAPH_FAILED)
        if os.environ.get("RDN_BENCH_DRY_HANG") == str(rank):   # tests of the deadline: this rank never returns
            while True:
                time.sleep(60)
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": world, "graph": args.graph,
                          "master_addr": os.environ.get("MASTER_ADDR"), "master_port": os.environ.get("MASTER_PORT"),
                          "launched_by": "bench.py" if os.environ.get("RDN_BENCH_LAUNCHED") else "external"}),
              flush=True)
        return
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cpu_group = None   # host-side agreement between the ranks (gloo), beside RCCL
    if world > 1:
        if args.dist_backend == "nccl":
            from vub_image_denoising_amd.ddp import capture_safe_env
            capture_safe_env()   # (RCCL inside the captured train step)
            dist.init_process_group("nccl", device_id=dev)
            cpu_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group("gloo")

    def all_ranks_ok(ok):
        """Every rank's flag, agreed over the host-side group (never over RCCL, whose
        state a failed capture may have left behind)."""
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=cpu_group)
        return bool(t.item())

    graph = args.graph == "on" and not args.pmc_child
    own_launcher = bool(os.environ.get("RDN_BENCH_LAUNCHED"))
    capture_err = None
    try:
        tr = Trainer(dev, args.batch, args.size, args.base_filters, args.dtype, rank, world, graph=graph)
    except GraphCaptureError as e:
        capture_err = e
        tr = e.trainer
        _log(f"rank {rank}: graph capture failed ({e.__cause__!r})")
    if world > 1 and graph and not all_ranks_ok(capture_err is None):
        # the hipGraph capture of the data-parallel step raised on some rank: no rank may
        # replay alone, and the RCCL communicator is suspect after a failed capture (a
        # capture that failed after some collectives were enqueued can leave the ranks'
        # op counts mismatched, and the first eager all-reduce would hang until the
        # watchdog).  Every rank exits EXIT_GRAPH_FAILED under every launcher: bench's own
        # launcher restarts the job eagerly from fresh processes; under torchrun, rerun
        # with --graph off
        _log(f"rank {rank}: a rank's capture failed; exiting (rerun with --graph off under an external launcher)"
             if not own_launcher else f"rank {rank}: a rank's capture failed; the launcher restarts eagerly")
        dist.destroy_process_group()
        sys.exit(EXIT_GRAPH_FAILED)
    elif capture_err is not None:
        raise capture_err
    graph = tr.graph is not None
    for i in range(args.warmup):
        if graph and world > 1 and i == 0:
            # the first replay of the RCCL step: a failure here ends this rank with
            # EXIT_GRAPH_FAILED under every launcher (its peers are left inside the
            # replay's collectives; bench's launcher restarts the job eagerly, torchrun
            # stops the job), never a silent eager fallback in a suspect process
            try:
                tr.step(i)
                torch.cuda.synchronize()
            except Exception as e:   # noqa: BLE001
                _log(f"rank {rank}: first replay of the captured RCCL step failed ({e!r})")
                sys.stderr.flush()
                os._exit(EXIT_GRAPH_FAILED)
            continue
        tr.step(i)
    torch.cuda.synchronize()

    # per-kernel profile pass (not timed): find the dominant kernel instantiation
    # (backward serialised: every launch timed alone, not beside the other stream)
    profs = [tr.profile() for _ in range(PROFILE_PASSES)]
    prof = profs[0]
    table = prof.summary()
    dom = max(table, key=lambda k: table[k]["ms"])
    if rank == 0 and args.layer_report:
        with open(args.layer_report, "w") as f:
            json.dump({k: {kk: (sorted(vv) if isinstance(vv, set) else vv) for kk, vv in d.items()}
                       for k, d in sorted(table.items(), key=lambda kv: -kv[1]["ms"])}, f, indent=1)
        with open(args.layer_report.replace(".json", "_per_layer.json"), "w") as f:
            json.dump(prof.per_layer(), f, indent=0)

    # timed region.  Eager: events around the dominant kernel's launches inside it.
    # Graph: the replays are timed; the dominant kernel's launch times come from an
    # eager pass of the same steps right after (events cannot be timed inside a replay)
    live = EventTracer(keys={dom})
    sync = getattr(tr.unet._rdn_flat, "grad_sync", None) if world > 1 else None
    if graph:
        el, loss = tr.timed(args.steps, world, None)
        if sync is not None:
            sync.timing = []   # (events only in the eager pass: a replay cannot be timed inside)
        el_eager, _ = tr.timed(args.steps, world, live)
    else:
        if sync is not None:
            sync.timing = []
        el, loss = tr.timed(args.steps, world, live)
        el_eager = el
    exposed = exposed_graph = None

    def over_ranks(mine, note):
        ex = torch.zeros(world, dtype=torch.float64)
        ex[rank] = -1.0 if mine is None else mine
        dist.all_reduce(ex, group=cpu_group)   # (each rank fills its own slot)
        per = [None if v < 0 else round(v, 4) for v in ex.tolist()]
        vals = [v for v in per if v is not None]
        return {"per_rank": per, "max": max(vals) if vals else None,
                "mean": round(sum(vals) / len(vals), 4) if vals else None, "unit": "ms per step", "note": note}
    if sync is not None:
        mine = sync.exposed_ms()
        sync.timing = None
        exposed = over_ranks(mine, "eager pass of the timed steps: end of the last gradient bucket's all-reduce "
                                   "on the comm stream minus the end of the backward on the compute stream "
                                   "(0 when hidden)")
        if graph and sync.stamps is not None:
            # the replayed step itself: its GradSync stamp kernels, read after each of
            # `steps` further (untimed) replays
            from vub_image_denoising_amd import _hip as H
            from vub_image_denoising_amd.ddp import exposure_from_stamps
            samples = []
            for i in range(args.steps):
                tr.step(i)
                torch.cuda.synchronize()
                samples.append(sync.stamps.tolist())
            st = exposure_from_stamps(samples, H.lib().rdn_wall_clock_khz())
            exposed_graph = over_ranks(None if st is None else st["mean"],
                                       "hipGraph replays of the timed step: device-clock stamps on the compute "
                                       "stream before and after its wait on the last all-reduce, less the launch "
                                       "gap of two back-to-back stamps (ddp.exposure_from_stamps)")
    if world > 1:
        tt = torch.tensor([el, el_eager], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el, el_eager = tt.tolist()
    loss_v = loss.item()
    d = live.summary()[dom]
    host_ms = tr.host_issue_ms() if world == 1 else None
    tr.eager = True
    host_eager_ms = tr.host_issue_ms() if (world == 1 and graph) else host_ms
    tr.eager = False

    if rank == 0:
        images = args.batch * world * args.steps
        avg_ms = d["ms"] / d["n"]
        flops_per = d["flops"] / d["n"]
        bytes_per = d["bytes"] / d["n"]
        peak_mfma = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        t_mfma = flops_per / (peak_mfma * 1e12)
        t_hbm = bytes_per / (PEAK_HBM_GBS * 1e9)
        if t_mfma >= t_hbm:
            roof = {"bound": "mfma", "achieved": round(flops_per / (avg_ms * 1e-3) / 1e12, 2), "peak": peak_mfma,
                    "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": round(bytes_per / (avg_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof["traffic"] = None
        if not (args.no_traffic or args.pmc_child) and world == 1:
            _log(f"PMC traffic passes for {dom}")
            traffic, note = pmc_traffic(dom, args)
            if traffic is not None:
                roof["traffic"] = round(traffic / 1e6, 3)
                roof["traffic_unit"] = "MB per launch"
                roof["algorithmic_bytes_mb"] = round(bytes_per / 1e6, 3)
                roof["traffic_over_algorithmic"] = round(traffic / bytes_per, 3)
            roof["traffic_source"] = note
        roof["kernel"] = dom
        roof["avg_launch_us"] = round(avg_ms * 1e3, 2)
        # the same kernel timed alone (profiling pass, serialised backward): the
        # timed region overlaps weight-gradient launches with the dgrad chain, so
        # a launch there shares the CUs with the other stream
        iso_ms = table[dom]["ms"] / table[dom]["n"]
        roof["isolated_avg_launch_us"] = round(iso_ms * 1e3, 2)
        roof["isolated_frac"] = round((flops_per / (iso_ms * 1e-3) / 1e12 / peak_mfma) if roof["bound"] == "mfma"
                                      else (bytes_per / (iso_ms * 1e-3) / 1e9 / PEAK_HBM_GBS), 4)
        roof["launches_per_step"] = d["n"] // args.steps
        roof["share_of_step"] = round(d["ms"] / (el_eager * 1e3), 4)
        roof[f"dense_conv_path_b{args.batch}"] = dense_conv_path_median(profs, args.batch)
        extra = None
        if world == 1 and not (args.no_extra or args.pmc_child):
            del tr
            torch.cuda.empty_cache()
            extra = extra_configs(dev, args)
            roof["dense_conv_path"] = extra["b32"].pop("dense_conv_path")
        want_cpu = world == 1 and not (args.no_cpu_baseline or args.pmc_child)   # rank 0 at N = 1 only
        if want_cpu:
            _log("CPU baseline")
        cpu = cpu_baseline(args.cpu_seconds, args.batch, args.size) if want_cpu else None
        infer = None
        if not (args.no_inference or args.pmc_child) and world == 1:
            _log("sampler measurements")
            infer = inference_bench(dev, args.base_filters)
            _log("config 1 forward (CPU oracle and GPU)")
            infer["config1_rdunet64_forward"] = config1_forward(dev)
            _log("RDUNet(128) forward on 1x3x256x256")
            infer["rdunet128_forward_256"] = rdunet128_forward(dev)
        out = {
            "metric": "images/sec (256x256x3) RDUNet diffusion train step",
            "value": round(images / el, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 3),
            "execution": "hipGraph replay per step" if graph else "eager launches",
            "eager_ms_per_step": round(el_eager * 1e3 / args.steps, 3),
            "host_issue_ms_per_step": host_ms,
            "eager_host_issue_ms_per_step": host_eager_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded U(-1,1) clean + Gaussian sigma in {15,25,50}/255*2, resident in HBM)",
            "config": {"workload": "RDUNet_T(base_filters=%d) diffusion train step, fwd+Charbonnier+bwd+clip+AdamW"
                                   % args.base_filters,
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "image": [3, args.size, args.size], "timesteps": 20,
                       "parallelism": f"dp{world}", "optimizer_step": "every step",
                       "launcher": ("single process" if world == 1 else
                                    "bench.py child processes" if os.environ.get("RDN_BENCH_LAUNCHED") else
                                    "external (torchrun)"),
                       "dist_backend": (args.dist_backend if world > 1 else None),
                       "final_loss": round(loss_v, 5)},
            "b32_images_per_s": extra["b32"]["images_per_s"] if extra else None,
            "fp32_images_per_s": extra["fp32"]["images_per_s"] if extra else None,
            "extra_configs": extra,
            "roofline": roof,
            "exposed_allreduce_ms": exposed,
            "exposed_allreduce_ms_graph": exposed_graph,
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
            "cpu_baseline": cpu,
            "inference": infer,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
