"""loner_amd — MI355X-native implicit-map optimisation path for LONER (esulimma/LONER @ 2024_08_07).

Product package.  Hot path = hand-written HIP kernels for gfx950 behind the C ABI in
``include/loner_amd.h`` (``loner_amd/_lib/libloner_amd.so``), bound with ctypes in ``_lib``.
Host-side mirrors of the reference interface:
  tcnn       tinycudann-compatible Encoding / Network / NetworkWithInputEncoding
  nerf       DecoupledNeRF                      (src/models/nerf_tcnn.py)
  rendering  render_rays / raw2outputs / ...    (src/models/rendering_tcnn.py)
  sampling   UniformRaySampler / OccGridRaySampler (src/models/ray_sampling.py)
  model      Model / OccupancyGridModel         (src/models/model_tcnn.py)
  optimizer  Optimizer (fused step)             (src/mapping/optimizer.py)
  step       FieldState / StepEngine: the fused optimiser step
  rays       world cube + LiDAR ray building    (src/common/ray_utils.py, pose_utils.py)
  synthetic  synthetic LiDAR scenes for the benchmark configs C1-C5
"""
__version__ = "0.1.0"
