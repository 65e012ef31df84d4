"""CPU oracle for the LONER implicit-map optimisation path — TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference algorithm (esulimma/LONER @ 2024_08_07)
used *only* as a checker: by ``tests/``, by ``__graft_entry__.smoke()`` and by the
``cpu_baseline`` leg of ``bench.py``.  Nothing in the product package ``loner_amd`` imports it,
and the product path fails loudly when its HIP extension is missing instead of falling back here.

Pinning:
  * rendering / sampling / loss / OGM / ray building are pinned against golden vectors produced
    by importing the reference's own pure-torch functions in the build container
    (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``);
  * the hash-grid encoding and the fully-fused MLP live in tiny-cuda-nn v1.7 (``README.md:343``),
    which is absent from ``/root/reference`` and CUDA-only: their restatement follows tcnn v1.7's
    published algorithm and is **parity unpinned** against tcnn itself (known-answer tests only).

Modules
  rng       counter-based RNG shared bit-exactly with the HIP kernels
  hashgrid  tcnn v1.7 HashGrid (levels, dense/hash index, trilinear fwd, scatter bwd)
  mlp       tcnn FullyFusedMLP (no bias, ReLU, fp16 weights/activations, padded output)
  render    linspace, samplers, sample_pdf, grid_sample, raw2outputs (default + adjusted) fwd/bwd
  loss      JS divergence, get_weights_gt, LiDAR loss fwd + analytic grads, OGM logits grad
  optim     torch.optim.Adam and OGM SGD restatements
  rays      get_far_val, build_lidar_rays, compute_world_cube
  step      one full optimiser step composed from the above (CPU baseline + end-to-end parity)
"""
