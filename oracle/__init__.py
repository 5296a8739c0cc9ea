"""CPU oracle for the diffusion-RDUNet hot path — TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product package ``vub_image_denoising_amd`` never imports anything
from here and fails loudly when its HIP library is missing.

Contents
--------
* ``weights``     — portable counter-hash parameter generator (splitmix64 +
                    Box-Muller, numpy) so fixtures never need a weight file.
* ``rdunet_ref``  — fp32/fp64 restatement of the reference network, loss,
                    train step and samplers with ``torch.nn.functional`` on the
                    CPU (NCHW/OIHW, the same aten math the reference runs).

Parity pinning: the restatement is checked against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` → ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.
"""
