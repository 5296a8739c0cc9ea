"""Per-launch A/B of the gate-out epilogue: every finisher input gradient of the B16
256^2 bf16 train step timed with its gate-out fields set and cleared (plus the
separate rdn_prelu_bwd pass the gate-out replaces), interleaved in one process.

    python scripts/gate_kbench.py [out.json]
"""
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import vub_image_denoising_amd as vm
    from vub_image_denoising_amd import _hip as H
    from vub_image_denoising_amd import engine as E
    E.GATE_OUT = True   # (off by default in the step)
    torch.manual_seed(0)
    m = vm.RDUNet_T(base_filters=32).cuda()
    m.set_compute_dtype("bf16")
    x = torch.rand(16, 3, 256, 256, device="cuda") * 2 - 1
    t = torch.rand(16, 1, 1, 1, device="cuda")
    y = m(x, t)
    y.square().mean().backward()
    torch.cuda.synchronize()
    eng = next(iter(m._rdn_engines.values()))[0]
    lib = H.lib()
    st = torch.cuda.current_stream()

    def timed(fn, reps=20):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return 1e3 * s.elapsed_time(e) / reps

    rows = []
    for J in eng.layers:
        K = J.extra.get("gates")
        if K is None:
            continue
        d_go = J.dgrad_desc
        d_no = H.ConvDesc.from_buffer_copy(d_go)
        d_no.gout = d_no.gout_pre = d_no.gout_alpha = d_no.gout_part = None
        d_no.gout_ps = d_no.gout_pre_ps = d_no.gout_c0 = 0
        olvl = eng._out_level(K)
        n, h, w = eng.grid[olvl]
        P = eng.P[olvl]
        pre = eng.bufs[K.pre]
        dd = eng._slice(K.ddst)
        dyp, pws = K.extra["dyp"], K.extra["pws"]
        alpha = eng.named[K.act + ".weight"].data_ptr()

        def prelu():
            H.check(lib.rdn_prelu_bwd(eng.code, P, n, h, w, K.cout, K.cout_pad, dd[0], dd[1], dd[2], dd[3], None,
                                      pre.data_ptr(), pre.shape[1], alpha, dyp, None, None, pws, st.cuda_stream),
                    "prelu")

        r = {"finisher": J.name, "gated": K.name}
        for rep in range(2):   # interleaved
            r.setdefault("go_us", []).append(timed(lambda: H.check(lib.rdn_conv_fwd(C.byref(d_go), st.cuda_stream))))
            r.setdefault("plain_us", []).append(timed(lambda: H.check(lib.rdn_conv_fwd(C.byref(d_no), st.cuda_stream))))
            r.setdefault("prelu_us", []).append(timed(prelu))
        r = {k: (round(min(v), 2) if isinstance(v, list) else v) for k, v in r.items()}
        r["kernel"] = eng._kernel_key(d_go)
        r["delta_us"] = round(r["go_us"] - r["plain_us"] - r["prelu_us"], 2)
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot = {k: round(sum(r[k] for r in rows), 1) for k in ("go_us", "plain_us", "prelu_us", "delta_us")}
    print(json.dumps({"total": tot}))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump({"rows": rows, "total": tot}, f, indent=1)


if __name__ == "__main__":
    main()
