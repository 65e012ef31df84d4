/* loner_amd.h — C ABI of the MI355X-native LONER implicit-map optimisation path.
 *
 * Every entry point replaces one piece of the reference's sigma-field step
 * (esulimma/LONER @ 2024_08_07; file:line relative to /root/reference):
 *
 *   lnr_hashgrid_fwd/_bwd(_rays)  tinycudann HashGrid encode used by
 *                                 tcnn.NetworkWithInputEncoding  src/models/nerf_tcnn.py:35-38,68/71
 *                                 and tcnn.Encoding              src/models/nerf_tcnn.py:40,64
 *   lnr_sigma_mlp_fwd/_bwd        tcnn FullyFusedMLP (32->64 ReLU->1, no bias)
 *                                 src/models/nerf_tcnn.py:35-38, cfg/nerf_config/default_nerf_hash.yaml:26-31
 *   lnr_sample_ogm / _uniform     OccGridRaySampler / UniformRaySampler + sample_pdf
 *                                 src/models/ray_sampling.py:18-92, src/models/rendering_tcnn.py:19-68
 *   lnr_composite                 raw2outputs / raw2outputs_adjusted src/models/rendering_tcnn.py:70-295
 *   lnr_composite_loss_bwd        compute_loss (LiDAR branch) + autograd through raw2outputs
 *                                 src/mapping/optimizer.py:701-859, src/models/losses.py:29-51
 *   lnr_field_train               fused sigma MLP fwd + composite + loss + composite bwd + MLP bwd
 *                                 (the body of one optimiser step, src/mapping/optimizer.py:436-450)
 *   lnr_loss_finalize             scalar loss / mean depth-eps from per-ray partials (optimizer.py:767,838-844)
 *   lnr_adam_step                 torch.optim.Adam step on the flat params  src/mapping/optimizer.py:255-265,460
 *   lnr_hashgrid_bwd_rays_jac_adam  the table's backward with that Adam step fused in (optimizer.py:450,460)
 *   lnr_ogm_update                Optimizer._step_occupancy_grid  src/mapping/optimizer.py:897-908
 *   lnr_rgb_render                colour head (SH4 + 2^19 HashGrid + FullyFusedMLP) + colour map
 *                                 src/models/nerf_tcnn.py:80-95, src/models/rendering_tcnn.py:283-289
 *   lnr_rgb_train / lnr_build_camera_rays  colour-head training (camera phase)
 *                                 src/mapping/optimizer.py:541-688,861-894, src/common/ray_utils.py:175-212
 *   lnr_motion_compensate / lnr_sky_rays  per-keyframe scan preprocessing
 *                                 src/common/sensors.py:169-231, examples/fdt_optimize_implicit_map_utils.py:38-77
 *   lnr_build_lidar_rays          per-step ray selection (RANDOM / MASK / sky) + KeyFrame.build_lidar_rays
 *                                 src/mapping/optimizer.py:363-424, src/mapping/keyframe.py:75-105,
 *                                 src/common/ray_utils.py:31-60,269-322
 *
 * Conventions:
 *   - all data pointers are DEVICE pointers owned by the caller (PyTorch); no allocation, no host
 *     synchronisation inside any call; every call only enqueues work on `stream` (a hipStream_t,
 *     NULL = default stream) and is safe to capture in a hipGraph;
 *   - return 0 (LNR_OK) or a negative error code; lnr_last_error() returns a thread-local message;
 *   - stateless and re-entrant.
 *
 * Layouts:
 *   rays     (R, 13) fp32  [o(3) d(3) viewdir(3) 0 0 near far]   src/common/ray_utils.py:314-317
 *   z        (R, S)  fp32  sorted sample depths (normalised units)
 *   table    (n_entries, 2) fp16 forward shadow; fp32 master/grad/m/v in the optimiser
 *   enc      "level-major": element (sample n, level l) at enc[l * enc_stride + n], one half2
 *            (uint32) per element; enc_stride >= N.  The tcnn-compatible AoS layout (N, 2L) is
 *            produced by lnr_enc_to_aos.
 *   d_enc    same indexing, one float2 per element
 *   mlp      sigma MLP weights, row-major [out][in] per layer: W0 (64,32) then W1 (16,64); fp16
 */
#ifndef LONER_AMD_H
#define LONER_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LNR_OK 0
#define LNR_ERR_ARG (-1)
#define LNR_ERR_HIP (-2)

#define LNR_MAX_LEVELS 32

const char* lnr_last_error(void);
int lnr_version(void);

/* ---------------------------------------------------------------- per-step scalars (graph replay) */
/* The scalars that change from one optimiser step to the next, in DEVICE memory, so that a step
 * captured once in a hipGraph replays with the current step's values (no kernel argument changes).
 * Every entry point that takes `dev_step` (or a struct holding it) reads these fields from it when it
 * is not NULL, in place of the corresponding host argument:
 *   key             the draw key (lnr_step_key(seed, global_step)): lnr_sample_ogm / _uniform, the
 *                   ray build (lnr_ray_window.dev_step), the sigma noise (lnr_loss_params.dev_step)
 *   los_lambda      lnr_loss_params.los_lambda (optimizer.py:712-716, decayed on global_step + 1)
 *   los_eps         lnr_loss_params.los_eps (optimizer.py:781-785)
 *   adam_step_size  lr / (1 - beta1^t), adam_bc2_sqrt = sqrt(1 - beta2^t): lnr_adam_step(_ranges)
 *                   (lnr_adam_coefficients forms both exactly as those calls do from step and lr) */
typedef struct lnr_step_scalars {
  uint32_t key;
  float los_lambda;
  float los_eps;
  float adam_step_size;
  float adam_bc2_sqrt;
  uint32_t pad[3];
} lnr_step_scalars;
/* dev[0..n) = values[0..n) (n <= 4 HOST structs, carried as the kernel's argument), enqueued on `stream`:
 * the launch before a captured step's replay sets that step's scalars (and the next step's, for its
 * prefetched ray build and sampling) in stream order. */
int lnr_step_scalars_set(const lnr_step_scalars* values, int32_t n, lnr_step_scalars* dev, void* stream);
/* Host: the fp32 Adam coefficients lnr_adam_step forms for 1-based step t and learning rate lr. */
int lnr_adam_coefficients(int32_t step, double lr, double beta1, double beta2, float* step_size, float* bc2_sqrt);

/* ---------------------------------------------------------------- hash grid */
typedef struct lnr_grid_desc {
  uint32_t n_levels;          /* tcnn "n_levels" */
  uint32_t n_features;        /* tcnn "n_features_per_level"; must be 2 */
  uint32_t log2_hashmap_size; /* tcnn "log2_hashmap_size" */
  uint32_t base_resolution;   /* tcnn "base_resolution" */
  float per_level_scale;      /* tcnn "per_level_scale" (default 2.0) */
  uint32_t n_entries;         /* sum of level sizes */
  float scale[LNR_MAX_LEVELS];
  uint32_t resolution[LNR_MAX_LEVELS];
  uint32_t size[LNR_MAX_LEVELS];
  uint32_t offset[LNR_MAX_LEVELS + 1];
} lnr_grid_desc;

/* Fill `d` exactly as tcnn v1.7's GridEncodingTemplated constructor lays the levels out. */
int lnr_grid_desc_init(lnr_grid_desc* d, uint32_t n_levels, uint32_t n_features, uint32_t log2_hashmap_size,
                       uint32_t base_resolution, float per_level_scale);

/* pos01 (N,3) fp32 in [0,1]^3 -> enc (level-major half2).  tcnn Encoding forward.
 * bwd_ws (optional, may be NULL): the backward workspace of the SAME positions; when given, the
 * forward also records the backward's per-block record histogram, so a following backward can be
 * called with LNR_BWD_COUNTS_READY and skips its counting pass. */
int lnr_hashgrid_fwd(const lnr_grid_desc* d, const float* pos01, int64_t n, const uint16_t* table,
                     uint32_t* enc, int64_t enc_stride, void* bwd_ws, int64_t bwd_ws_bytes, void* stream);
/* Positions generated from rays and samples: pos01 = (o + d*z + 1) / 2 (nerf_tcnn.py:63). */
int lnr_hashgrid_fwd_rays(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                          int32_t n_samples, const uint16_t* table, uint32_t* enc, int64_t enc_stride,
                          void* bwd_ws, int64_t bwd_ws_bytes, void* stream);
/* Early ray termination, the encode of one phase: samples [lo, hi) (multiples of 64; n_samples % 64 == 0) of
 * the rays ray_list[0 .. *ray_count) (DEVICE; ray_list NULL: every ray), as lnr_hashgrid_fwd_rays encodes them;
 * the other samples' encodings are left unwritten.  bwd_ws (the first phase only, lo == 0, every ray): the
 * backward's record histogram of EVERY sample, as lnr_hashgrid_fwd_rays records it, for a full backward with
 * LNR_BWD_COUNTS_READY (the live backward counts its own).  Without bwd_ws only the listed rays' phase samples
 * are encoded, by a grid that leaves at once past the list's end.  expect_rays: the caller's estimate of
 * *ray_count (0: none); a small one selects a grid for a sparse phase (one level per workgroup, walking the
 * listed rows).  Every grid encodes exactly the listed rays' samples, whatever the count.  See
 * lnr_field_sigma_phase. */
int lnr_hashgrid_fwd_rays_phase(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                int32_t n_samples, const uint16_t* table, uint32_t* enc, int64_t enc_stride,
                                void* bwd_ws, int64_t bwd_ws_bytes, const uint32_t* ray_list,
                                const uint32_t* ray_count, int64_t expect_rays, int32_t lo, int32_t hi,
                                void* stream);
/* Forward of samples whose compositing weight can be zero (the colour head: rgb = sum w_i c_i + ...,
 * rendering_tcnn.py:286): samples with live[n] == 0 (exactly) issue no gathers, every other sample is
 * encoded exactly as lnr_hashgrid_fwd_rays does.  A dead sample gets a zero encoding when its aligned
 * 16-sample tile (n / 16) holds a live sample; the encodings of a tile with no live sample are left
 * unwritten (lnr_rgb_render and lnr_rgb_train skip such tiles).  live = the (R,S) weights of the sigma
 * pass.  No backward histogram. */
int lnr_hashgrid_fwd_rays_live(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                               int32_t n_samples, const uint16_t* table, const float* live, uint32_t* enc,
                               int64_t enc_stride, void* stream);
/* lnr_hashgrid_fwd_rays_live that also records the backward's histogram in `bwd_ws` (as
 * lnr_hashgrid_fwd_rays does), counting a sample with live[n] == 0 at the coherent levels only (its
 * zero gradient merges into the runs there) and not at the others: the records of
 * lnr_hashgrid_bwd_rays_live, which can then be called with LNR_BWD_COUNTS_READY (no counting pass). */
int lnr_hashgrid_fwd_rays_live_ws(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                  int32_t n_samples, const uint16_t* table, const float* live, uint32_t* enc,
                                  int64_t enc_stride, void* bwd_ws, int64_t bwd_ws_bytes, void* stream);
/* Backward: d_table (n_entries,2) fp32 = scatter of corner weights * d_enc, as an atomic-free
 * binned scatter of 8-byte records (fp16 values at a per-level power-of-two scale from max |d_enc|)
 * with int64 fixed-point accumulation at a unit that depends on N alone.  d_table is OVERWRITTEN (every entry, zero where
 * no sample touches it, all zero for N = 0) and the result is bitwise reproducible; `workspace` holds
 * at least lnr_hashgrid_bwd_workspace_bytes(d, N) bytes.
 * Input gradient (tcnn's backward w.r.t. the positions, src/models/nerf_tcnn.py:63,68-71 when pos
 * requires grad, e.g. joint pose + map optimisation, src/mapping/optimizer.py:256-262): when d_pos is
 * not NULL, d_pos (N,3) fp32 = dL/dpos01 (OVERWRITTEN): per sample, the sum over (level, feature) of
 * d_enc * d enc / d pos01, the trilinear blend's derivative from the fp16 `table` (the forward's
 * operand, 4-byte aligned): tcnn v1.7 kernel_grid's dy_dx + kernel_grid_backward_input.  The _rays
 * forms give it per sample w.r.t. pos01 = (o + d z + 1) / 2.  Deterministic (one fixed-order sum per
 * sample).  d_table may be NULL (no table gradient: workspace unused), d_pos may be NULL (table unused),
 * not both.  The input gradient is its own launch, so a call without d_pos costs nothing extra. */
#define LNR_BWD_COUNTS_READY 1
#define LNR_BWD_NO_ACCUM 2      /* stop after the scatter: lnr_hashgrid_bwd_accum then finishes level ranges */
#define LNR_BWD_LEVEL_MAX_READY 4 /* the caller stored max |d_enc| per level at lnr_hashgrid_bwd_level_max():
                                     no pass over d_enc for it.  The maxima may be rank-local under data
                                     parallelism: they only pick each level's power-of-two record scale,
                                     fp16 rounding is scale-invariant, and the fixed-point unit sits far
                                     below what reaches Adam */
#define LNR_BWD_PREPARE_ONLY 16   /* stop before the scatter: the live records' histogram (or, with
                                     LNR_BWD_COUNTS_READY, the forward's) scanned into bucket offsets; needs
                                     LNR_BWD_LIVE or LNR_BWD_COUNTS_READY (reads d_sigma, not J) */
#define LNR_BWD_PREPARED 32       /* a LNR_BWD_PREPARE_ONLY call with the same arguments ran: scatter + accumulate */
#define LNR_BWD_LIVE 8            /* lnr_hashgrid_bwd_rays_jac(_adam): the live backward.  A sample with
                                     d_sigma[n] == 0 (relu(sigma + noise) = 0 or transmittance 0,
                                     rendering_tcnn.py:252-266) adds exactly 0 to every entry, so only samples with
                                     d_sigma != 0 emit records (coherent levels: only runs holding one), after its
                                     own histogram pass over those samples (a forward histogram is not needed and,
                                     with LNR_BWD_COUNTS_READY, not read).  The fixed-point unit depends on N alone,
                                     so d_table is BITWISE the full backward's.  Pays when most samples are dead (a
                                     trained field: ~89 % at C2); ignored where the level-looped scatter does not
                                     apply (small batches, other grids). */
int64_t lnr_hashgrid_bwd_workspace_bytes(const lnr_grid_desc* d, int64_t n);
/* Device address of the n_levels per-level max |d_enc| floats inside `workspace` (the same for
 * every n: the workspace's first bytes). */
float* lnr_hashgrid_bwd_level_max(const lnr_grid_desc* d, int64_t n, void* workspace);
/* Device address of the last backward's bucket segment starts inside `workspace` (n_buckets + 1 uint64,
 * buckets = the levels' 4096-entry table chunks in level order; the last is the number of records the
 * scatter placed): for tests and tools that measure the record volume (e.g. of the live backward). */
const uint64_t* lnr_hashgrid_bwd_seg_start(const lnr_grid_desc* d, int64_t n, void* workspace);
int lnr_hashgrid_bwd(const lnr_grid_desc* d, const float* pos01, int64_t n, const float* d_enc,
                     int64_t enc_stride, float* d_table, const uint16_t* table, float* d_pos, void* workspace,
                     int64_t workspace_bytes, int32_t flags, void* stream);
int lnr_hashgrid_bwd_rays(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                          int32_t n_samples, const float* d_enc, int64_t enc_stride, float* d_table,
                          const uint16_t* table, float* d_pos, void* workspace, int64_t workspace_bytes,
                          int32_t flags, void* stream);
/* The table gradient of samples with a live mask (the colour grid: live = the compositing weights, d_enc
 * of a weight-0 sample is 0): at the levels that are not coherent, samples with live[n] == 0 emit no records
 * (the others emit theirs, zero or not).  Bitwise the same d_table as lnr_hashgrid_bwd_rays (records of zero
 * add nothing and the fixed-point unit does not follow the record counts).  With LNR_BWD_COUNTS_READY the histogram must come from
 * lnr_hashgrid_fwd_rays_live_ws with the same mask. */
int lnr_hashgrid_bwd_rays_live(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                               int32_t n_samples, const float* d_enc, int64_t enc_stride, const float* live,
                               float* d_table, void* workspace, int64_t workspace_bytes, int32_t flags,
                               void* stream);
/* The same, from lnr_field_train's compact encoding gradient: d_enc = d_sigma[n] * J[l][n] with J
 * level-major fp16 pairs (one uint32 per level and sample, level stride jac_stride). */
int lnr_hashgrid_bwd_rays_jac(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                              int32_t n_samples, const uint32_t* d_jac, const float* d_sigma, int64_t jac_stride,
                              float* d_table, const uint16_t* table, float* d_pos, void* workspace,
                              int64_t workspace_bytes, int32_t flags, void* stream);
/* The same with Adam fused in: where the backward finishes a table entry's gradient it applies
 * torch.optim.Adam's update to that parameter (the arithmetic of lnr_adam_step, so the parameters,
 * moments and fp16 shadow come out bitwise equal) instead of storing the gradient, for the
 * 2 * n_entries table parameters at the head of `param`, `shadow`, `m`, `v`.  The step's Adam on the
 * parameters after the table (the MLP) stays a lnr_adam_step.  N = 0 is Adam with a zero gradient.
 * LNR_BWD_NO_ACCUM is refused (a gradient exchanged between ranks must reach memory first). */
typedef struct lnr_adam_epilogue {
  float* param;
  uint16_t* shadow;
  float* m;
  float* v;
  int32_t step;  /* 1-based, as lnr_adam_step */
  double lr, beta1, beta2, eps;
  const lnr_step_scalars* dev_step; /* non-NULL: step size and bias correction from device memory */
} lnr_adam_epilogue;
int lnr_hashgrid_bwd_rays_jac_adam(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                   int32_t n_samples, const uint32_t* d_jac, const float* d_sigma, int64_t jac_stride,
                                   const lnr_adam_epilogue* adam, void* workspace, int64_t workspace_bytes,
                                   int32_t flags, void* stream);
/* With flags & LNR_BWD_NO_ACCUM the three calls above stop after the scatter; this finishes the
 * levels [level_begin, level_end) (n = samples of that call, same workspace): their slice of
 * d_table is final on return, so a data-parallel caller can all-reduce it while the next range
 * accumulates. */
int lnr_hashgrid_bwd_accum(const lnr_grid_desc* d, int64_t n, void* workspace, int64_t workspace_bytes,
                           uint32_t level_begin, uint32_t level_end, float* d_table, void* stream);
/* The same after a live backward (flags: the backward's LNR_BWD_LIVE): picks the accumulation for its smaller
 * record counts (the unit work list); the result is the same either way. */
int lnr_hashgrid_bwd_accum_flags(const lnr_grid_desc* d, int64_t n, void* workspace, int64_t workspace_bytes,
                                 uint32_t level_begin, uint32_t level_end, float* d_table, int32_t flags, void* stream);
/* Same result with one fp32 atomic pair per corner (coarse levels merged in-wave); d_table
 * accumulates.  Kept as an independent implementation for cross-checking and A/B timing. */
int lnr_hashgrid_bwd_atomic(const lnr_grid_desc* d, const float* pos01, int64_t n, const float* d_enc,
                            int64_t enc_stride, float* d_table, void* stream);
int lnr_hashgrid_bwd_rays_atomic(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                 int32_t n_samples, const float* d_enc, int64_t enc_stride, float* d_table,
                                 void* stream);
/* level-major half2 -> tcnn AoS (N, 2L) fp16, and AoS fp16/fp32 grads -> level-major float2. */
int lnr_enc_to_aos(const uint32_t* enc, int64_t enc_stride, int64_t n, uint32_t n_levels, uint16_t* out, void* stream);
int lnr_aos_grad_to_enc(const uint16_t* g_aos_f16, const float* g_aos_f32, int64_t n, uint32_t n_levels,
                        float* d_enc, int64_t enc_stride, void* stream);

/* tcnn "SphericalHarmonics" encoding (colour head, nerf_tcnn.py:43,86): dir01 (N,3) fp32 in [0,1]^3
 * -> out (N, degree^2) fp16 row-major.  degree 1..4 (LONER uses 4). */
int lnr_sh_encode(const float* dir01, int64_t n, int32_t degree, uint16_t* out, void* stream);

/* ---------------------------------------------------------------- sigma MLP */
#define LNR_SIGMA_W0 (64 * 32)
#define LNR_SIGMA_W1 (16 * 64)
#define LNR_SIGMA_MLP_PARAMS (LNR_SIGMA_W0 + LNR_SIGMA_W1)

/* sigma (N) fp16 = MLP(enc).  Non-finite outputs are clamped to +-65504 (nerf_tcnn.py:74-78). */
int lnr_sigma_mlp_fwd(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, int64_t n, uint16_t* sigma,
                      void* stream);
/* Number of fp32 words of workspace lnr_sigma_mlp_bwd / lnr_field_train need for dW slabs. */
int64_t lnr_dw_workspace_words(int64_t n_rows);
/* d_sigma (N) fp32 -> d_enc (level-major float2, overwritten) and d_w (3072 fp32, ACCUMULATED). */
int lnr_sigma_mlp_bwd(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, int64_t n, const float* d_sigma,
                      float* d_enc, float* d_w, float* workspace, void* stream);

/* ---------------------------------------------------------------- sampling */
/* Random draws: when u_* is NULL, draws come from the counter-based generator keyed by `key`
 * (see lnr_step_key) and the GLOBAL ray index ray_offset + r, so a sharded batch draws exactly
 * what the unsharded batch draws.  Otherwise u_jitter is (R, S/2) and u_pdf is (R, S/2). */
uint32_t lnr_step_key(uint32_t seed, uint32_t step);
int lnr_sample_ogm(const float* rays, int64_t n_rays, int32_t n_samples, const float* occ, int32_t occ_res,
                   float perturb, const float* u_jitter, const float* u_pdf, uint32_t key, int64_t ray_offset,
                   float* z, const lnr_step_scalars* dev_step, void* stream);
int lnr_sample_uniform(const float* rays, int64_t n_rays, int32_t n_samples, float perturb, const float* u_jitter,
                       uint32_t key, int64_t ray_offset, float* z, const lnr_step_scalars* dev_step, void* stream);

/* ---------------------------------------------------------------- compositing + loss */
#define LNR_RENDER_DEFAULT 0
#define LNR_RENDER_ADJUSTED 1

#define LNR_LOSS_L1_JS 0
#define LNR_LOSS_L2_JS 1
#define LNR_LOSS_L1_LOS 2
#define LNR_LOSS_L2_LOS 3

typedef struct lnr_loss_params {
  int32_t kind;            /* LNR_LOSS_* (optimizer.py:757-791) */
  float scale;             /* world-cube scale factor (metres per normalised unit) */
  float los_lambda;        /* already decayed for this global step (optimizer.py:712-716) */
  float depthloss_lambda;  /* loss.depthloss_lambda */
  float min_depth_eps;     /* loss.min_depth_eps */
  float min_js, max_js, js_alpha; /* loss.JS_loss */
  float los_eps;           /* L*_LOS only: decayed depth_eps for this iteration (optimizer.py:781-785) */
  float far_ref;           /* far bound of GLOBAL ray 0: optimizer.py:724 compares every ray with it */
  float inv_n_opaque;      /* 1 / (global opaque-ray count) */
  float inv_rs;            /* 1 / (global rays * samples) */
  const float* dev_n_opaque; /* optional DEVICE scalar: global opaque count (e.g. after an all-reduce);
                                when non-NULL it overrides inv_n_opaque (= 1/max(count,1)) */
  const float* dev_far_ref;  /* optional DEVICE scalar overriding far_ref (rays built on the device:
                                lnr_build_lidar_rays writes it) */
  uint32_t* dev_status;      /* optional DEVICE word: LNR_STATUS_* bits are OR-ed in (no host sync; the
                                caller reads it when it chooses, e.g. once per window) */
  float* dev_loss_out;       /* optional DEVICE [8]: lnr_field_train also writes lnr_loss_finalize's output
                                here, in its last launch (one launch less per step) */
  int32_t flags;             /* LNR_LP_* */
  const lnr_step_scalars* dev_step; /* optional DEVICE: key (the noise), los_lambda and los_eps from here */
  float* dev_d_ray;          /* optional DEVICE (R,2), lnr_field_train: [dL/d|d|, dL/dfar] per ray, the loss's
                                dependence on the ray itself when the poses are optimised (optimizer.py:258-262;
                                rendering_tcnn.py:248,274-278; the samples z are detached, ray_sampling.py:75-90).
                                With the hash grid's input gradient (lnr_hashgrid_bwd_rays_jac's d_pos) it gives
                                dL/d{origin, direction, far} of every ray (joint pose + map) */
  uint32_t* dev_term_hist;   /* optional DEVICE LNR_TERM_HIST_SLOTS x (n_samples / 64 + 1) counters, slot-major,
                                lnr_field_train with n_samples a multiple of 64: ray r adds 1 to bin c / 64 of slot
                                r mod LNR_TERM_HIST_SLOTS, c = the number of its samples after which its
                                transmittance product is still >= LNR_ERT_T_MIN (c = n_samples: it never terminates).
                                The caller sums the slots (they only spread the atomics) and differences two reads:
                                the library never clears them.  The rays alive after sample k (a multiple of 64)
                                are the bins >= k / 64, which is what picks the phases of
                                lnr_hashgrid_fwd_rays_phase / lnr_field_sigma_phase */
} lnr_loss_params;
#define LNR_TERM_HIST_SLOTS 256
#define LNR_ERT_T_MIN 1e-50      /* early ray termination: a ray whose transmittance product fell below this has
                                    float transmittance exactly 0 at every later sample (csrc/field.hip) */
#define LNR_LP_DW_OVERWRITE 1  /* lnr_field_train STORES d_w (the MLP gradient) instead of adding to it */
#define LNR_LP_SIGMA_READY 2   /* lnr_field_train: sigma is already in its workspace (lnr_field_sigma_phase), the
                                  MLP forward is not run again (n_samples in {64, 128, 256, 512}) */
#define LNR_LP_FORWARD_ONLY 4  /* lnr_field_train (n_samples in {64, 128, 256, 512}, d_enc_jac): the sigma forward and
                                  the compositing + loss + its backward only (dL/dsigma in the workspace); a second
                                  call with the same arguments and LNR_LP_BACKWARD_ONLY runs the MLP backward and the
                                  reductions.  Between the two, work that needs dL/dsigma but not J (the live
                                  backward's LNR_BWD_PREPARE_ONLY) can run on another stream */
#define LNR_LP_BACKWARD_ONLY 8

/* Status bits (replace the reference's per-step host checks):
 *   LNR_STATUS_NAN_LOSS     loss is NaN: optimizer.py:854 asserts "NaN Loss Encountered"
 *   LNR_STATUS_INF_LOSS     loss is +-inf
 *   LNR_STATUS_SIGMA_CLIPPED a sigma was non-finite and clipped by nan_to_num (nerf_tcnn.py:74-78 warns) */
#define LNR_STATUS_NAN_LOSS 1u
#define LNR_STATUS_INF_LOSS 2u
#define LNR_STATUS_SIGMA_CLIPPED 4u
#define LNR_STATUS_NONFINITE_OUTPUT 8u  /* lnr_status_scan found nan/inf (rendering_tcnn.py:419-424 DEBUG scan) */
/* ORs `bit` into the device word `status` when any of values[0..n) is nan or inf (no host sync). */
int lnr_status_scan(const float* values, int64_t n, uint32_t bit, uint32_t* status, void* stream);

/* Per-ray partial sums written by the loss kernels: [depth_sq_err, los_sum, opacity_abs_err, eps, opaque] */
#define LNR_RAY_STATS 5

/* Forward compositing from given sigma (R,S) fp32 (fp16-valued) and noise (R,S) (NULL + noise_std>0 ->
 * generated; noise_std==0 -> none).  Outputs may be NULL except depth. */
int lnr_composite(const float* rays, const float* z, const float* sigma, int64_t n_rays, int32_t n_samples,
                  int32_t strategy, float noise_std, const float* noise, uint32_t key, int64_t ray_offset,
                  float* weights, float* depth, float* opacity, float* variance, void* stream);
/* Training loss + gradient from given sigma: d_sigma (R,S) fp32, ray_stats (R, LNR_RAY_STATS). */
int lnr_composite_loss_bwd(const float* rays, const float* z, const float* sigma, const float* depth_gt,
                           int64_t n_rays, int32_t n_samples, float noise_std, const float* noise, uint32_t key,
                           int64_t ray_offset, const lnr_loss_params* lp, float* weights, float* depth,
                           float* opacity, float* d_sigma, float* ray_stats, void* stream);
/* Autograd backward of lnr_composite (the tcnn-compatible render_rays path, where the loss is the
 * caller's torch code): d_sigma (R,S) fp32 from upstream gradients of weights (R,S), depth, opacity
 * and variance (R); any of them may be NULL (= zero).  Same noise arguments as the forward, so the
 * noise is regenerated bit-identically instead of being stored.  d_ray (optional, (R,2)): the
 * render's gradient w.r.t. the ray itself, [dL/d|d| (deltas are scaled by the direction's norm,
 * rendering_tcnn.py:248), dL/dfar (the default depth's far term, :274-278; 0 for the adjusted
 * strategy)] - what autograd returns when the rays require grad (poses under optimisation). */
int lnr_composite_bwd(const float* rays, const float* z, const float* sigma, int64_t n_rays, int32_t n_samples,
                      int32_t strategy, float noise_std, const float* noise, uint32_t key, int64_t ray_offset,
                      const float* g_weights, const float* g_depth, const float* g_opacity, const float* g_variance,
                      float* d_sigma, float* d_ray, void* stream);
/* Workspace (fp32 words) lnr_field_train needs: the dW slabs, then an (n_rays, n_samples) d_sigma
 * buffer between its ray phase and its tile-parallel MLP backward. */
int64_t lnr_field_train_workspace_words(int64_t n_rays, int32_t n_samples);
/* Fused: sigma MLP forward from enc, compositing, loss, compositing backward, MLP backward.
 * Writes d_enc (level-major float2), accumulates d_w (3072 fp32), per-ray stats; optional outputs NULL.
 * d_enc_level_max (optional, 16 floats): OVERWRITTEN with max |d_enc| per level, the hash-grid
 * backward's record scales (pass lnr_hashgrid_bwd_level_max(...) and LNR_BWD_LEVEL_MAX_READY).
 * d_enc_jac (optional; n_samples 64, 128, 256 or 512): written INSTEAD of d_enc (which may be NULL):
 * J = d sigma / d enc as level-major fp16 pairs, one uint32 per (level, sample), so that
 * d_enc = d_sigma * J with d_sigma the (n_rays, n_samples) fp32 dL/dsigma this call leaves at
 * workspace + lnr_dw_workspace_words(n_rays); lnr_hashgrid_bwd_rays_jac takes both (half the bytes).
 * J is written only for the 32-sample tile pairs holding a sample with d_sigma != 0: elsewhere d_enc is 0
 * whatever J is, and the J entries keep stale values (every consumer of the pair forms d_sigma * J as 0 where
 * d_sigma == 0).  The MLP gradient is bitwise the one with every pair computed (a dead pair adds exact zeros).
 * workspace: lnr_field_train_workspace_words(n_rays, n_samples) fp32 words. */
int lnr_field_train(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays, const float* z,
                    const float* depth_gt, int64_t n_rays, int32_t n_samples, float noise_std, const float* noise,
                    uint32_t key, int64_t ray_offset, const lnr_loss_params* lp, float* d_enc, float* d_w,
                    float* workspace, float* ray_stats, float* depth, float* opacity, float* weights,
                    float* d_enc_level_max, uint32_t* d_enc_jac, void* stream);
/* Early ray termination (the training step on a trained field): the sigma MLP forward of samples [lo, hi) of
 * the rays list_in[0 .. *count_in) (DEVICE; ignored when lo == 0: every ray) (multiples of 64) into
 * lnr_field_train's workspace, where lnr_field_train with LNR_LP_SIGMA_READY reads it.  When hi < n_samples it
 * then takes each listed ray's transmittance[r] (fp64; 1 before lo == 0) times the
 * product over the phase of s = 1 - alpha + 1e-10 (the compositing's own arithmetic: noise, deltas as
 * lnr_field_train draws them; key, noise_std, noise, ray_offset, lp->dev_step as there), and lists the rays whose
 * product stays >= LNR_ERT_T_MIN in list_out[0 .. *count_out) in list order (through `scratch`, at least
 * n_rays 32-bit words); the others get sigma 0 at their samples [hi, n_samples).  A ray whose product fell below
 * 1e-50 has every later
 * sample's float transmittance exactly 0 in the compositing, so its later samples' sigma and encodings cannot
 * change any output: the phases lnr_hashgrid_fwd_rays_phase -> lnr_field_sigma_phase, phase by phase (the lists
 * alternating between two buffers), then lnr_field_train with LNR_LP_SIGMA_READY, give the step's results without
 * evaluating them (csrc/field.hip).
 * lp: optional (dev_status: LNR_STATUS_SIGMA_CLIPPED for the evaluated samples; dev_step: the key). */
int lnr_field_sigma_phase(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays,
                          const float* z, int64_t n_rays, int32_t n_samples, int32_t lo, int32_t hi, float noise_std,
                          const float* noise, uint32_t key, int64_t ray_offset, const lnr_loss_params* lp,
                          float* workspace, const uint32_t* list_in, const uint32_t* count_in, uint32_t* list_out,
                          uint32_t* count_out, double* transmittance, void* scratch, void* stream);
/* Joint pose + map (optimizer.py:235-262): the per-keyframe gradient of the pose tensors [t, axis-angle] (K, 6)
 * from a step's per-sample dL/dpos01 d_pos (n_rays * n_samples, 3) (lnr_hashgrid_bwd_rays_jac) and per-ray
 * [dL/d|d|, dL/dfar] d_ray (n_rays, 2) (lnr_loss_params.dev_d_ray), for rays built as
 * LidarRayDirections.build_lidar_rays builds them (o = (t + shift) / scale, d = R v / |R v|, far = min(r_max /
 * scale, get_far_val(o, d)); ray_utils.py:31-60,269-322): ray r is window slot slots[r] (slots NULL: slot0 + r),
 * of keyframe slot_kf[slot], and carries slot_pose[slot] (1: a LiDAR ray of an optimised pose, 0: a sky ray --
 * built from the detached pose, keyframe.py:98 -- or an anchored keyframe).  grad (K, 6) is OVERWRITTEN (a
 * fixed-order, deterministic sum); ray_ws: n_rays * 12 floats.  far_range = r_max / scale. */
int lnr_pose_grad(const float* rays, const float* z, const float* d_pos, const float* d_ray, int64_t n_rays,
                  int32_t n_samples, const int64_t* slots, int64_t slot0, const int32_t* slot_kf, const float* slot_pose,
                  const float* pose6, int32_t n_kf, float scale, float far_range, float* ray_ws, float* grad,
                  void* stream);
/* The poses' Adam step (torch.optim.Adam, the pose group of optimizer.py:262: betas, eps, lr = lrate_pose x the
 * ExponentialLR factor; step = this Adam's step count, from 1) on pose6 with moments m, v (K, 6), for keyframes
 * with optimise[k] != 0 (NULL: all), then rows (K, 12) = [R | t] of every pose (the RayWindow's pose layout; may
 * be NULL).  grad NULL: only the rows are written (m, v, step unused). */
int lnr_pose_adam(float* pose6, float* m, float* v, const float* grad, const uint8_t* optimise, int32_t n_kf,
                  int64_t step, float lr, float beta1, float beta2, float eps, float* rows, void* stream);
/* Forward-only render from enc (inference path, C3 shape): sigma MLP + compositing.  With weights
 * (R,S) given, the sigma MLP runs tile-parallel first and stages sigma in weights, which the
 * compositing then overwrites with the weights (weights must not alias the other buffers); without,
 * one fused kernel per ray.  Same results either way. */
int lnr_field_render(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays, const float* z,
                     int64_t n_rays, int32_t n_samples, int32_t strategy, float noise_std, const float* noise,
                     uint32_t key, int64_t ray_offset, float* depth, float* opacity, float* variance,
                     float* weights, void* stream);
/* Colour head forward + colour map (DecoupledNeRF colour branch nerf_tcnn.py:80-95, raw2outputs
 * rendering_tcnn.py:283-289): w_rgb = tcnn flat fp16 params of the 48 -> 64 x n_hidden_layers -> 3
 * FullyFusedMLP (1..4 hidden layers), enc_rgb = level-major colour hash-grid encodings (16 levels x 2),
 * weights (R,S) = the sigma pass's compositing weights (lnr_field_render).  Directions = rays[:, 6:9]
 * (SH degree 4 of (viewdir + 1) / 2).  rgb (R,3) = sum_i w_i sigmoid(c_i) + 1 - sum_i w_i. */
int lnr_rgb_render(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb, int64_t enc_stride,
                   const float* rays, const float* weights, int64_t n_rays, int32_t n_samples, float* rgb,
                   void* stream);
/* out[0] = loss, out[1] = mean eps, out[2..4] = depth/los/opacity terms, out[5] = opaque count,
 * from (R, LNR_RAY_STATS). */
int lnr_loss_finalize(const float* ray_stats, int64_t n_rays, const lnr_loss_params* lp, float* out, void* stream);

/* out[0] = number of opaque rays: depth_gt > 0 && !(depth_gt > far_ref) (optimizer.py:724-727).
 * dev_far_ref: optional DEVICE scalar overriding far_ref. */
int lnr_count_opaque(const float* depth_gt, int64_t n_rays, float far_ref, const float* dev_far_ref, float* out,
                     void* stream);

/* ---------------------------------------------------------------- ray selection + building */
#define LNR_SELECT_RANDOM 0 /* torch.randint over each scan (optimizer.py:365-366) */
#define LNR_SELECT_MASK 1   /* int(0.75 n) trunk points (0.5 < z_sensor < 8 m) + the rest from the other points,
                               each without replacement (optimizer.py:367-379) */
#define LNR_SELECT_ALL 2    /* every point of every scan, in order (LidarRayDirections.fetch_chunk_rays) */
#define LNR_SELECT_GIVEN 3  /* caller-supplied scan-local indices, one per slot (parity tests) */

/* The active keyframe window, resident on the device for the whole window.  All pointers are
 * DEVICE pointers; counts are validated by the caller (loner_amd.rays.RayWindow). */
typedef struct lnr_ray_window {
  int32_t n_kf;
  float scale;                /* WorldCube.scale_factor */
  float shift[3];             /* WorldCube.shift */
  float r_min, r_max;         /* ray_range (metres) */
  const float* poses;         /* [K][12]: the 3x4 [R | t] rows of each keyframe's lidar pose (world) */
  const float* dirs;          /* [P][3] sensor-frame ray directions (LidarScan.ray_directions, transposed) */
  const float* dists;         /* [P] ranges (metres) */
  const int32_t* scan_off;    /* [K+1] point offsets of each keyframe's scan in dirs / dists */
  const int32_t* order;       /* MASK: [P] per keyframe, scan-local indices of its trunk points, then the rest */
  const int32_t* n_trunk;     /* MASK: [K] trunk points per keyframe */
  const float* sky_dirs;      /* [Q][3] sky directions (LidarScan.sky_rays), or NULL without sky rays */
  const int32_t* sky_off;     /* [K+1] offsets into sky_dirs, or NULL */
  const int32_t* ray_off;     /* [K+1] output slots of each keyframe: its LiDAR rays, then its sky rays */
  const int32_t* n_sel;       /* [K] LiDAR slots per keyframe (slots beyond them are sky rays) */
  const int32_t* n_sel_trunk; /* MASK: [K] LiDAR slots drawn from the trunk points */
  const lnr_step_scalars* dev_step; /* optional DEVICE: the draw key from here instead of `key` */
} lnr_ray_window;

/* Build output slots [slot0, slot0 + n_slots) of the window's ray batch: rays (n_slots, 13), depth
 * (n_slots) normalised, valid (n_slots) = far > near + 1 m / scale (the reference drops invalid rays;
 * NULL allowed), point_index (n_slots) scan-local point of each slot (NULL allowed), far_ref (1) =
 * far bound of the first valid slot of the WHOLE batch (NULL allowed).  Draws keyed by
 * (key, keyframe, slot-in-keyframe): a sharded build reproduces the unsharded one slot for slot. */
int lnr_build_lidar_rays(const lnr_ray_window* window, int32_t select, const int32_t* given, uint32_t key,
                         int64_t slot0, int64_t n_slots, float* rays, float* depth, uint8_t* valid,
                         int32_t* point_index, float* far_ref, void* stream);

/* Camera rays (KeyFrame.build_camera_rays, src/mapping/keyframe.py:108-127 ->
 * CameraRayDirections.build_rays, src/common/ray_utils.py:175-212): for pixel p = j * width + i,
 * rays[k] = [o, d, -d, i, j, r_min / scale, get_far_val(o, d)] with d = normalise(R dirs[p]),
 * o = (t + shift) / scale; intensities[k] = image[p] (channels floats, optional).  dirs = the
 * (height * width, 3) undistorted camera-frame directions (get_ray_directions, ray_utils.py:62-124,
 * computed once per calibration by the host). */
typedef struct lnr_camera_desc {
  int32_t width, height, channels;
  float scale;        /* WorldCube.scale_factor */
  float shift[3];     /* WorldCube.shift */
  float r_min;        /* ray_range[0] (metres) */
  float pose[12];     /* camera pose in the world, 3x4 [R | t] rows */
} lnr_camera_desc;
int lnr_build_camera_rays(const lnr_camera_desc* cam, const float* dirs, const float* image, const int64_t* pixels,
                          int64_t n, float* rays, float* intensities, void* stream);
/* A whole camera window in one launch: frames = DEVICE array of n_frames {camera, image}; frame f
 * fills slots [f n_per_frame, (f + 1) n_per_frame) from pixels[f stride + first + j] (a window's
 * per-frame pixel schedules, optimizer.py:626-644).  intensities may be NULL. */
typedef struct lnr_camera_frame {
  lnr_camera_desc cam;
  const float* image;   /* (height * width, channels) fp32, DEVICE */
} lnr_camera_frame;
int lnr_build_camera_rays_window(const lnr_camera_frame* frames, int32_t n_frames, const float* dirs,
                                 const int64_t* pixels, int64_t stride, int64_t first, int64_t n_per_frame,
                                 float* rays, float* intensities, void* stream);

/* Colour-head training, camera phase (Optimizer._do_iterate_optimizer_camera + compute_loss_camera,
 * src/mapping/optimizer.py:541-688,861-894): sigma frozen and detached (weights = the sigma pass's
 * compositing weights, lnr_field_render); rgb as lnr_rgb_render; loss = l1(rgb, intensities) as a
 * mean over the 3 * (global) rays: inv_count = 1 / (3 n_rays_global).  Writes rgb (R,3), loss[0]
 * (optional; local rays only), d_enc (level-major float2, the colour-grid backward's input, as
 * lnr_field_train's) and d_w (OVERWRITTEN: the colour MLP's weight gradient, tcnn flat layout,
 * lnr_rgb_mlp_params floats).  Deterministic (fixed-order slab reduction).  d_enc_level_max
 * (optional, 16 floats): OVERWRITTEN with max |d_enc| per level, as lnr_field_train's (pass
 * lnr_hashgrid_bwd_level_max(...) and LNR_BWD_LEVEL_MAX_READY to the colour grid's backward). */
int64_t lnr_rgb_mlp_params(int32_t n_hidden_layers);
int64_t lnr_rgb_train_workspace_bytes(int32_t n_hidden_layers, int64_t n_rays);
int lnr_rgb_train(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb, int64_t enc_stride,
                  const float* rays, const float* weights, const float* intensities, int64_t n_rays,
                  int32_t n_samples, float inv_count, float* rgb, float* loss, float* d_enc, float* d_w,
                  void* workspace, int64_t workspace_bytes, float* d_enc_level_max, void* stream);

/* ---------------------------------------------------------------- optimiser */
/* torch.optim.Adam (no weight decay); step is 1-based.  shadow (fp16) may be NULL.  dev_step (optional):
 * the step size and bias correction from there (step and lr are then ignored). */
int lnr_adam_step(float* param, uint16_t* shadow, const float* grad, float* m, float* v, int64_t n, int32_t step,
                  double lr, double beta1, double beta2, double eps, const lnr_step_scalars* dev_step, void* stream);
/* The same step over up to LNR_ADAM_MAX_RANGES independent ranges in one launch (the sharded
 * optimiser's per-level-range chunks, loner_amd.step.StepEngine(zero=...)). */
#define LNR_ADAM_MAX_RANGES 8
typedef struct lnr_adam_range {
  float* param;
  uint16_t* shadow; /* may be NULL */
  const float* grad;
  float* m;
  float* v;
  int64_t n;
} lnr_adam_range;
int lnr_adam_step_ranges(const lnr_adam_range* ranges, int32_t n_ranges, int32_t step, double lr, double beta1,
                         double beta2, double eps, const lnr_step_scalars* dev_step, void* stream);
/* OGM update: occ (res^3) -= lr * grid_sample^T(logits_grad(z*scale - depth_gt*scale)).  grad_ws is
 * workspace of ws_words fp32 (lnr_ogm_workspace_words(occ_res) for full speed; at least 3 res^3):
 * the splat accumulates in int64 fixed point in replicas of the grid that spread same-voxel
 * atomics (bitwise reproducible), and grad_ws[0, res^3) receives the fp32 gradient. */
int64_t lnr_ogm_workspace_words(int32_t occ_res);
int lnr_ogm_update(const float* rays, const float* z, const float* depth_gt, int64_t n_rays, int32_t n_samples,
                   float scale, float lr, float* occ, float* grad_ws, int64_t ws_words, int32_t occ_res, void* stream);

/* Split form for data-parallel runs: grad_ws[0:res^3] = grid_sample^T(logits_grad) (the call zeroes the
 * workspace), then occ -= lr * grad_ws[0:res^3] after the caller has all-reduced that slice. */
int lnr_ogm_grad(const float* rays, const float* z, const float* depth_gt, int64_t n_rays, int32_t n_samples,
                 float scale, float* grad_ws, int64_t ws_words, int32_t occ_res, void* stream);
int lnr_sgd_step(float* param, const float* grad, int64_t n, float lr, void* stream);

/* OccupancyGridModel.interpolate (src/models/model_tcnn.py:126-134) as an operator of its own, for the
 * module-level drop-in (Optimizer._step_occupancy_grid, src/mapping/optimizer.py:897-908, calls it and
 * backpropagates through it).  Replaces torch.nn.functional.grid_sample on a (1, 1, res, res, res) grid
 * with (n, 3) points in [-1, 1]: trilinear, align_corners=False, zeros padding.
 *   lnr_grid_sample3d      out[i] = grid_sample(grid, pts[i])
 *   lnr_grid_sample3d_bwd  dgrid = sum_i dout[i] d out[i] / d grid (overwritten; the points get no
 *                          gradient: the reference's points are detached).  Deterministic: int64
 *                          fixed point with a unit from max |dout| and n (about 2^-42 of max |dout|
 *                          per point at n = 10^6); ws: lnr_grid_sample3d_bwd_workspace_words(res)
 *                          fp32 words, 8-byte aligned (2 + 2 res^3 at least). */
int lnr_grid_sample3d(const float* grid, int32_t res, const float* pts, int64_t n, float* out, void* stream);
int64_t lnr_grid_sample3d_bwd_workspace_words(int32_t res);
int lnr_grid_sample3d_bwd(const float* pts, const float* dout, int64_t n, int32_t res, float* dgrid, float* ws,
                          int64_t ws_words, void* stream);

/* ---------------------------------------------------------------- per-keyframe scan preprocessing */
/* LidarScan.motion_compensate (src/common/sensors.py:169-231).  Host-computed per scan: the start pose
 * rotation (row-major) and translation, end - start translation, axis/angle of R_start^T R_end
 * (identity = angle < 1e-9), timestamps t0/t1 of the two poses, and the first 3 rows of
 * inv(T_world_to_target).  dirs (P,3) / dists (P) are rewritten in place. */
typedef struct lnr_motion_comp {
  float start_rot[9];
  float start_t[3];
  float delta_t[3];
  float axis[3];
  float angle;
  float t0, t1;
  float target_inv[12];
  int32_t identity;
} lnr_motion_comp;
int lnr_motion_compensate(const lnr_motion_comp* mc, const float* timestamps, float* dirs, float* dists,
                          int64_t n_points, void* stream);

/* compute_sky_rays (examples/fdt_optimize_implicit_map_utils.py:38-77): sky directions (rotated by
 * rot, the lidar pose rotation, row-major) of one scan's dirs (P,3), written as (count, 3) into out
 * (capacity cap directions, lnr_sky_rays_capacity() is enough); count (1 int32, device) = number. */
typedef struct lnr_sky_params {
  float rot[9];
  int32_t top_rows;     /* TOP_ROWS = 3 */
  float horizon_deg;    /* HORIZON_OFFSET = 10 */
} lnr_sky_params;
int64_t lnr_sky_rays_capacity(void);
int lnr_sky_rays(const float* dirs, int64_t n_points, const lnr_sky_params* params, float* out, int64_t cap,
                 int32_t* count, void* stream);

/* ---------------------------------------------------------------- utilities */
/* dst[i] = lo + (hi-lo) * U(splitmix64(((uint64)seed << 32) + start + i)) */
int lnr_fill_uniform(float* dst, int64_t n, uint32_t seed, float lo, float hi, int64_t start, void* stream);
int lnr_f32_to_f16(const float* src, uint16_t* dst, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LONER_AMD_H */
