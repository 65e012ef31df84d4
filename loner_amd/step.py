"""Fused optimiser step on the HIP C-ABI: the MI355X-native body of
``Optimizer._do_iterate_optimizer``'s step loop (src/mapping/optimizer.py:354-475).

One step = OGM sampling -> hash-grid encode -> fused [sigma MLP, compositing, LiDAR loss,
compositing backward, MLP backward] -> hash-grid backward -> (all-reduce) -> Adam
[-> OGM update every ``N_iters_acc`` global steps, checked before the increment as at
optimizer.py:466-469].  All buffers are allocated once; a step only enqueues kernels on the
current stream (no host synchronisation) and can be captured in a HIP graph.

Parameter layout (tcnn ``NetworkWithInputEncoding``: network first, then encoding):
    params[0:3072]            sigma MLP, W0 (64,32) then W1 (16,64), row-major [out][in]
    params[3072:]             hash table, (n_entries, 2), level-major
fp32 master + Adam moments; an fp16 shadow of the whole buffer feeds the forward kernels.
"""
import math
import os
import warnings
from dataclasses import dataclass, field

import torch

from . import _lib as L


@dataclass
class LossConfig:
    """``model_config.loss`` (cfg/model_config/default_model_config.yaml:40-60)."""
    loss_selection: str = "L1_JS"
    min_js_score: float = 1.0
    max_js_score: float = 10.0
    js_alpha: float = 1.0
    decay_los_lambda: bool = False
    los_lambda: float = 1000.0
    min_los_lambda: float = 10.0
    los_lambda_decay_rate: float = 0.001
    los_lambda_decay_steps: float = 15000
    decay_depth_eps: bool = True
    depth_eps: float = 3.0
    min_depth_eps: float = 0.5
    depth_eps_decay_rate: float = 0.95
    depth_eps_decay_steps: float = 1
    depthloss_lambda: float = 0.005

    @staticmethod
    def from_dict(d):
        js = d.get("JS_loss", {})
        keys = {k: d[k] for k in LossConfig.__dataclass_fields__ if k in d}
        return LossConfig(**keys, min_js_score=js.get("min_js_score", 1.0), max_js_score=js.get("max_js_score", 10.0),
                          js_alpha=js.get("alpha", 1.0))

    def los_lambda_at(self, global_step):
        # optimizer.py:712-716 (and :846-848): decay evaluated on global_step + 1
        if self.decay_los_lambda:
            return max(self.los_lambda * (self.los_lambda_decay_rate ** ((global_step + 1) / self.los_lambda_decay_steps)),
                       self.min_los_lambda)
        return self.los_lambda

    def los_eps_at(self, iteration_idx):
        # optimizer.py:781-785
        if self.decay_depth_eps:
            return max(self.depth_eps * (self.depth_eps_decay_rate ** (iteration_idx / self.depth_eps_decay_steps)),
                       self.min_depth_eps)
        return self.depth_eps


@dataclass
class StepConfig:
    n_samples: int = 512              # render.N_samples_train
    perturb: float = 1.0              # render.perturb
    raw_noise_std: float = 1.0        # render.raw_noise_std
    lr: float = 0.01                  # train.lrate_sigma_mlp
    occ_res: int = 100                # occ_model.voxel_size
    occ_lr: float = 1e-4              # occ_model.lr
    n_iters_acc: int = 10             # occ_model.N_iters_acc
    sampler: str = "OGM"              # samples_selection.strategy
    n_levels: int = 16
    log2_hashmap_size: int = 18
    base_resolution: int = 16
    per_level_scale: float = 2.0
    loss: LossConfig = field(default_factory=LossConfig)


class FieldState:
    """Parameters, Adam moments, fp16 shadow and the occupancy grid, resident on one GPU.

    With a data-parallel or sharded ``StepEngine`` on this state, the last step's OGM update and shadow
    all-gathers may still be pending on the device: call the engine's ``finish()`` (or ``drop_prefetch()`` /
    ``release()``, which call it) before reading ``occ``, ``shadow`` or ``state_dict()`` directly."""

    def __init__(self, cfg: StepConfig, device="cuda", seed=1337, table_init=1e-4):
        self.cfg = cfg
        self.device = torch.device(device)
        self.desc = L.grid_desc(cfg.n_levels, 2, cfg.log2_hashmap_size, cfg.base_resolution, cfg.per_level_scale)
        self.n_entries = int(self.desc.n_entries)
        self.n_mlp = L.SIGMA_MLP_PARAMS
        self.n_params = self.n_mlp + 2 * self.n_entries
        self.n_padded = (self.n_params + 3) // 4 * 4
        dev = self.device
        self.params = torch.zeros(self.n_padded, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.shadow = torch.zeros(self.n_padded, dtype=torch.float16, device=dev)
        self.occ = torch.zeros(cfg.occ_res ** 3, dtype=torch.float32, device=dev)
        self.occ_ws = torch.zeros(int(L.lib().lnr_ogm_workspace_words(cfg.occ_res)), dtype=torch.float32, device=dev)
        self.adam_step = 0
        # whether grad_table holds the last step's table gradient: a step with the table's Adam fused into
        # the backward (StepEngine.fused_adam) applies it where it is accumulated and never stores it
        self.grad_table_current = True
        self.init_params(seed, table_init)

    # tcnn init: FullyFusedMLP xavier-uniform per matrix, HashGrid U(-1e-4, 1e-4) (restated with a
    # counter-based generator: tcnn's PCG stream is not reproducible here)
    def init_params(self, seed=1337, table_init=1e-4):
        s = L.stream(self.device)
        a0 = math.sqrt(6.0 / (32 + 64))
        a1 = math.sqrt(6.0 / (64 + 16))
        p = self.params
        L.call("lnr_fill_uniform", (p), 64 * 32, seed, -a0, a0, 0, s)
        L.call("lnr_fill_uniform", L.ctypes.c_void_p(p.data_ptr() + 4 * 64 * 32), 16 * 64, seed + 1, -a1, a1, 0, s)
        L.call("lnr_fill_uniform", L.ctypes.c_void_p(p.data_ptr() + 4 * self.n_mlp), 2 * self.n_entries, seed + 2,
               -table_init, table_init, 0, s)
        self.refresh_shadow()

    def refresh_shadow(self):
        L.call("lnr_f32_to_f16", (self.params), (self.shadow), self.n_padded, L.stream(self.device))

    def reset_optimizer(self):
        """A new torch.optim.Adam per window / iteration config (optimizer.py:255-265)."""
        self.m.zero_()
        self.v.zero_()
        self.adam_step = 0

    # views
    @property
    def mlp_f16(self):
        return self.shadow[:self.n_mlp]

    @property
    def table_f16(self):
        return self.shadow[self.n_mlp:self.n_mlp + 2 * self.n_entries]

    @property
    def grad_table(self):
        """The table's slice of the flat gradient (the backward's output buffer).  NOT written by a step whose
        table Adam is fused into the backward (``grad_table_current`` is then False and the slice keeps an
        older gradient); use ``table_gradient()`` to read it safely."""
        return self.grad[self.n_mlp:self.n_mlp + 2 * self.n_entries]

    def table_gradient(self):
        """The last step's table gradient; raises when that step fused the table's Adam into the backward
        (the gradient never went to memory: run with StepEngine.fused_adam = False to keep it)."""
        if not self.grad_table_current:
            raise RuntimeError("the last step fused the table's Adam into the backward: its table gradient was "
                               "never stored (StepEngine.fused_adam = False keeps it)")
        return self.grad_table

    @property
    def grad_mlp(self):
        return self.grad[:self.n_mlp]

    def state_dict(self):
        return {"params": self.params[:self.n_params].clone(), "occupancy_grid": self.occ.clone(),
                "adam_step": self.adam_step, "m": self.m[:self.n_params].clone(), "v": self.v[:self.n_params].clone()}

    def load_state_dict(self, sd):
        self.params[:self.n_params].copy_(sd["params"])
        self.occ.copy_(sd["occupancy_grid"].reshape(-1))
        if "m" in sd:
            self.m[:self.n_params].copy_(sd["m"])
            self.v[:self.n_params].copy_(sd["v"])
            self.adam_step = int(sd.get("adam_step", 0))
        self.refresh_shadow()


FUSED_ADAM_MAX_N = 1 << 17  # samples up to which the step fuses the table's Adam into the backward ("auto")
# the level at which the two gradient-exchange ranges split: [cut, L) first, then [0, cut) + MLP.  Modelled per
# cut from the measured per-range accumulate at C4 shard 1/8 (tools/zero_tail_model.py): the
# exchange's critical path is 3 us shorter at 6 than at 4 and 13-20 us shorter than at 8 (round 4's cut) for
# ring bandwidths of 100-400 GB/s
AR_CUT_DEFAULT = 6
# with the sharded optimiser's all-gathers on a communicator of their own (bench.py LONER_EXCHANGE_GROUPS=2), the
# gather of range 1 overlaps range 2's reduce-scatter, and the model puts the best cut at 8 (levels 8-15 first):
# 168 us exposed at 200 GB/s if the two share the link bandwidth, 148 us if not, against 191 / 156 at cut 6
# (tools/zero_tail_model.py, profiles/r06_zero_tail_model_C4s8.txt)
AR_CUT_TWO_GROUPS = 8

# Early ray termination's cost model (us; csrc/field.hip, lnr_hashgrid_fwd_rays_phase + lnr_field_sigma_phase),
# fitted to round 6's kernel traces of the trained C2 step: the encode + sigma of one
# ray-sample ERT_SAMPLE_NS, phased or not; going phased ERT_FIXED_US; every phase after the first ERT_PHASE_US (its
# encode, sigma and list launches, latency-bound when few rays are left)
ERT_SAMPLE_NS, ERT_FIXED_US, ERT_PHASE_US = 0.150, 5.0, 28.0
TERM_HIST_SLOTS = 256  # LNR_TERM_HIST_SLOTS
ERT_MAX_CUTS = 4
ERT_MARGIN = 0.02  # eager steps: a plan replaces the current one only when modelled this much faster (of the full
# encode); under graph replay a new plan waits for the window's captures and takes no margin (StepEngine.ert_probe)


def ert_alive(hist, S):
    """From a termination histogram (lnr_loss_params.dev_term_hist: bin c // 64 per ray, c its samples before the
    transmittance product drops below LNR_ERT_T_MIN): the share of rays still alive after sample 64 k, k = 0..S/64."""
    import numpy as np
    h = np.asarray(hist, dtype=np.float64)
    tot = h.sum()
    if tot <= 0:
        return np.ones(S // 64 + 1)
    tail = np.cumsum(h[::-1])[::-1]  # rays with bin >= k
    return tail / tot


def ert_cost_us(bounds, alive, S, n_samples):
    """Modelled encode + sigma time of one step (n_samples ray-samples) with the phases ``bounds``
    ([0, c1, .., S]) or, for None, without early ray termination."""
    full = ERT_SAMPLE_NS * 1e-3 * n_samples
    if bounds is None:
        return full
    t = ERT_FIXED_US + ERT_PHASE_US * (len(bounds) - 2)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        t += full * float(alive[lo // 64]) * (hi - lo) / S
    return t


def ert_plan(hist, S, n_samples, current=None, max_cuts=ERT_MAX_CUTS, margin=ERT_MARGIN):
    """The early-ray-termination phases for the coming steps from the last steps' termination histogram: the
    cheapest under ert_cost_us among no termination and every set of at most ``max_cuts`` cuts at multiples of
    64 samples, kept only if it beats ``current`` (the plan in use: bounds or None) by ``margin`` of the full
    encode (so the graphs, captured per plan, are not re-captured for noise).  Returns bounds or None."""
    import itertools
    if S % 64 or S < 128:
        return None
    alive = ert_alive(hist, S)
    full = ert_cost_us(None, alive, S, n_samples)
    pos = list(range(64, S, 64))
    best, best_t = None, full
    for k in range(1, min(max_cuts, len(pos)) + 1):
        for cuts in itertools.combinations(pos, k):
            b = [0, *cuts, S]
            t = ert_cost_us(b, alive, S, n_samples)
            if t < best_t:
                best, best_t = b, t
    cur_t = ert_cost_us(current, alive, S, n_samples)
    return best if best_t < cur_t - margin * full else current


class StepEngine:
    """Preallocated workspaces for a fixed ray-batch size; ``step`` runs one optimiser step."""

    def __init__(self, state: FieldState, n_rays: int, seed: int = 0, allreduce=None, ray_offset: int = 0,
                 count_in_forward: bool = True, zero=None, reduce_scatter=None, all_gather=None, ar_cut=None):
        self.state = state
        self.cfg = state.cfg
        self.n_rays = n_rays
        self.S = self.cfg.n_samples
        self.N = n_rays * self.S
        self.seed = seed
        self.ray_offset = ray_offset
        # True (default): the forward counts every sample's records (no extra pass).  False: the
        # backward counts after the MLP backward and skips samples whose gradient is exactly zero at
        # fine levels (relu(sigma + noise) = 0).  Measured at C2: the zero share is small once the
        # field has trained a few steps, and the extra count pass (d_enc reads) costs more than the
        # records it saves (3.35 vs 3.18 ms/step), so it is opt-in for sparse-gradient workloads.
        self.count_in_forward = count_in_forward
        self.lr_factor = 1.0  # ExponentialLR: the caller sets gamma^k (optimizer.py:262, stepped per iteration)
        self.status = torch.zeros(1, dtype=torch.int32, device=state.device)  # LNR_STATUS_* bits
        self._warned_clip = False
        # level ranges of the bucketed gradient all-reduce, finest first: the first range's exchange
        # overlaps the later range's accumulation.  Every range is its own accumulate + finalize
        # launch pair, and at world size 1 over RCCL (no peer traffic; tools/dp_overhead.py, round 3) the step
        # cost 2.18-2.25 ms with one range, 2.23-2.30 with two (levels 8-15, then 0-7 + the MLP)
        # and 2.41-2.44 with four, against 2.12 without the hook; two ranges hide about half of the
        # 29.7 MB exchange for a fraction of the four ranges' cost.  LONER_AR_BUCKETS = 1, 2 or 4.
        # With two ranges the cut level is LONER_AR_CUT (default AR_CUT_DEFAULT; the modelled exposure of
        # the sharded optimiser's tail per cut: DESIGN.md section 7, tools/zero_tail_model.py).
        nl = self.cfg.n_levels
        nbk = int(os.environ.get("LONER_AR_BUCKETS", "2"))
        if nbk <= 1:
            cuts = [nl, 0]
        elif nbk == 2:
            cut = int(os.environ.get("LONER_AR_CUT", str(AR_CUT_DEFAULT if ar_cut is None else ar_cut)))
            cuts = sorted({nl, min(max(cut, 1), max(nl - 1, 1)), 0}, reverse=True)
        else:
            cuts = sorted({nl, max(nl - 5, 1), max(nl - 10, 1), min(3, nl), 0}, reverse=True)
        self.ar_groups = [(cuts[i + 1], cuts[i]) for i in range(len(cuts) - 1)]
        # callable(tensor[, async_op]) summing in place across ranks (torch.distributed.all_reduce
        # semantics), or None
        self.allreduce = allreduce
        dev = state.device
        # Sharded optimiser (ZeRO-1): zero = (rank, world).  Each level range's gradient slice is
        # reduce-scattered instead of all-reduced (reduce_scatter(out, inp, async_op), the semantics of
        # torch.distributed.reduce_scatter_tensor), the rank runs Adam on its 1/world chunk of every range,
        # and the updated fp16 shadow chunks are all-gathered (all_gather(out, inp, async_op), as
        # all_gather_into_tensor).  The fp32 master and the moments stay current only on each chunk's
        # owner: sync_master() all-gathers the master (checkpoints).  With zero but no collectives (one
        # process), the step does one rank's share of Adam and nothing else: the per-rank work of an
        # N-GPU run, for measuring it on one GPU (bench.py --shard-of).
        self.zero = None
        if zero is not None:
            zr, zw = int(zero[0]), int(zero[1])
            if not 0 <= zr < zw:
                raise ValueError(f"zero=(rank, world) out of range: {zero}")
            self.zero = (zr, zw)
            self.reduce_scatter, self.all_gather = reduce_scatter, all_gather
            if zw > 1 and allreduce is not None and (reduce_scatter is None or all_gather is None):
                raise ValueError("a sharded optimiser over ranks needs reduce_scatter and all_gather hooks")
            self.zero_chunks = []  # per level range: (a0, a1, chunk), this rank owning [a0 + r c, a0 + (r+1) c)
            for l0, l1 in self.ar_groups:
                a0, a1 = self._ar_range(l0, l1)
                if (a1 - a0) % (4 * zw):
                    raise ValueError(f"levels [{l0}, {l1}) hold {a1 - a0} parameters, not a multiple of 4 x {zw} ranks "
                                     "(the sharded optimiser needs equal, 16-B aligned chunks)")
                self.zero_chunks.append((a0, a1, (a1 - a0) // zw))
            if len(self.zero_chunks) > L.ADAM_MAX_RANGES:
                raise ValueError(f"{len(self.zero_chunks)} level ranges: at most {L.ADAM_MAX_RANGES} (one Adam launch)")
            self.zero_grad = [torch.empty(c, dtype=torch.float32, device=dev) for _, _, c in self.zero_chunks]
        self._pending_shadow = []  # async all-gather works of the last sharded step (finish())
        # data-parallel OGM step: the grid gradient's all-reduce runs asynchronously and the SGD step that
        # consumes it is enqueued before the grid's next reader (the next step's sampler, or finish())
        self._pending_ogm = None
        self.z = torch.empty(n_rays, self.S, dtype=torch.float32, device=dev)
        self.enc = torch.empty(self.cfg.n_levels, self.N, dtype=torch.int32, device=dev)
        self.ws = torch.empty(L.lib().lnr_field_train_workspace_words(n_rays, self.S), dtype=torch.float32, device=dev)
        # the encoding gradient: compact (d sigma / d enc as fp16 pairs + dL/dsigma, 4 + 4/L B per sample and
        # level) where the field kernel's per-ray path supports it, else d_enc itself (float2)
        self.compact_denc = self.S in (64, 128, 256, 512)
        if self.compact_denc:
            self.d_jac = torch.empty(self.cfg.n_levels, self.N, dtype=torch.int32, device=dev)
            self.d_enc = None
        else:
            self.d_enc = torch.empty(self.cfg.n_levels, self.N, 2, dtype=torch.float32, device=dev)
        self._r_last = n_rays  # the last step's ray count (d_sigma's place in the workspace follows it)
        self.bwd_ws_bytes = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(L.ctypes.byref(state.desc), self.N))
        self.bwd_ws = torch.empty(self.bwd_ws_bytes, dtype=torch.uint8, device=dev)
        # the backward's per-level max |d_enc| (record scales), written by the field kernel's MLP backward
        self.level_max_ptr = L.ctypes.c_void_p(L.lib().lnr_hashgrid_bwd_level_max(L.ctypes.byref(state.desc), self.N,
                                                                                   L.ptr(self.bwd_ws)))
        self.stats = torch.zeros(n_rays, L.RAY_STATS, dtype=torch.float32, device=dev)
        self.depth = torch.empty(n_rays, dtype=torch.float32, device=dev)
        self.opacity = torch.empty(n_rays, dtype=torch.float32, device=dev)
        self.loss_out = torch.zeros(8, dtype=torch.float32, device=dev)
        self.n_opaque = torch.zeros(1, dtype=torch.float32, device=dev)
        # the opaque count (and its all-reduce) runs on a side stream, off the critical path: only the
        # field kernel needs it (forked after the rays exist, joined before the field kernel)
        self._side = torch.cuda.Stream(device=dev)
        self._fork, self._join = torch.cuda.Event(), torch.cuda.Event()
        # The live backward's histogram, scans and lists need dL/dsigma only, not the MLP backward's J: with
        # split_bwd (LONER_SPLIT_BWD, default 1) they run on a side stream beside the MLP backward
        # (lnr_field_train's LNR_LP_FORWARD_ONLY / BACKWARD_ONLY halves, the backward's LNR_BWD_PREPARE_ONLY /
        # PREPARED halves), captured as two branches of the step's graph; bitwise the one-stream step
        self.split_bwd = os.environ.get("LONER_SPLIT_BWD", "1") != "0"
        self._bside = torch.cuda.Stream(device=dev)
        self._bfork, self._bjoin = torch.cuda.Event(), torch.cuda.Event()
        # on-device ray building (step_window)
        self.rays = torch.empty(n_rays, 13, dtype=torch.float32, device=dev)
        self.depth_gt = torch.empty(n_rays, dtype=torch.float32, device=dev)
        self.ray_valid = torch.empty(n_rays, dtype=torch.uint8, device=dev)
        self.far_ref = torch.empty(1, dtype=torch.float32, device=dev)
        # step_window on windows whose rays can fail the 1 m filter: two ray buffers, the next step's
        # build + compaction prefetched on a side stream (``prefetch``)
        self.prefetch = os.environ.get("LONER_PREFETCH", "1") != "0"
        self._pf, self._pf_parity = None, 0
        self._pf_stream = torch.cuda.Stream(device=dev)
        self._pf_fork = torch.cuda.Event()
        self._pf_bufs = [dict(rays=torch.empty_like(self.rays), dgt=torch.empty_like(self.depth_gt),
                              valid=torch.empty_like(self.ray_valid), far=torch.empty_like(self.far_ref),
                              rays_c=torch.empty_like(self.rays), dgt_c=torch.empty_like(self.depth_gt))
                         for i in range(2)]
        # step_window on windows whose rays all pass the filter: step k + 1's ray build and sampling
        # enqueued on a side stream right after step k (two ray / depth buffers), so they run in the
        # holes step k leaves (the scatter's last round, the accumulate's tail) instead of at the head
        # of step k + 1 (``pipeline``; not when step k updates the OGM, which the sampler reads)
        self.pipeline = os.environ.get("LONER_PIPELINE", "1") != "0"
        # the single-GPU step's table Adam fused into the backward (lnr_hashgrid_bwd_rays_jac_adam, bitwise
        # the separate lnr_adam_step).  "auto" (default): for batches of at most 2^17 samples, whose
        # whole-bucket accumulation spreads the Adam work over a workgroup per bucket (C1 0.161 -> 0.152
        # ms); at C2 the record-balanced accumulation's bucket ends carry it less well (1.950 -> 1.958-
        # 1.989 ms), so there it stays a separate pass.  LONER_FUSED_ADAM=1 / 0 forces it on / off; the
        # data-parallel paths always exchange the gradient first.
        self.fused_adam = {"0": False, "1": True}.get(os.environ.get("LONER_FUSED_ADAM", "auto"), "auto")
        self._pp, self._pp_parity = None, 0
        self._pp_stream = torch.cuda.Stream(device=dev)
        self._pp_fork = torch.cuda.Event()
        # step_window on all-valid windows, single process: the whole step (ray build, sampling, encode,
        # field, backward, Adam, and the OGM update on its steps) captured once per (window, OGM or not)
        # in a HIP graph and replayed, its per-step scalars (key, loss scalars, Adam coefficients) set in
        # device memory by one small launch before each replay (``lnr_step_scalars``): one graph launch
        # in place of ~18 kernel launches (LONER_GRAPH=0 turns it off; the pipelined path then runs)
        # LONER_GRAPH: auto (default: batches of at most 2^18 samples, where the host's launch cost is a
        # visible share of the step; measured C1 0.161 against 0.163 ms eager on a fast host, 0.188 against
        # 0.236 on a slow one; and from 2^22 samples, where every kernel fills the chip, so the eager path's
        # next-step prefetch (the sampler: texture-addresser work) slows the encode beside it about as much
        # as it hides: C2 1.910-1.916 against 1.918-1.923 ms eager since round 5's lighter sampler, 2.040
        # against 2.016 before it.  In between, the prefetch fills what the smaller kernels leave idle: C4
        # shard 1/8 0.374-0.381 eager against 0.380-0.381), 1 always, 0 never
        g = os.environ.get("LONER_GRAPH", "auto")
        self.use_graph = (g == "1") or (g == "auto" and (self.N <= (1 << 18) or self.N >= (1 << 22)))
        # the graph step's lnr_step_scalars (32 B)
        self._dev_steps = torch.zeros(8, dtype=torch.int32, device=dev)
        self.dev_step = self._dev_steps
        self._dev_step = None
        self._graphs, self._graph_window = {}, None
        self._capture_stream = torch.cuda.Stream(device=dev)
        # The live backward (LNR_BWD_LIVE): a sample with dL/dsigma = 0 (relu(sigma + noise) = 0,
        # rendering_tcnn.py:260) adds exactly 0 to the table gradient, and on a trained field most samples are such
        # (~80 % at C2 after the driver's windows, bench.py --field trained; ~0 % in the first steps from init).
        # The live backward places records only for the others, after a histogram pass over them: bitwise the
        # full backward's gradient, so the choice is a matter of speed only.  Its work skips by 64-sample wave
        # (a wave without a live sample does nothing), and its histogram pass costs ~0.16 ms at C2 when every
        # wave is live (C2 backward 1.15 against 0.99 ms from init, 0.49 against 0.95 ms trained with 69 % of the
        # waves dead: break-even near 20 % dead waves).  LONER_LIVE_BWD: 1 always, 0 never, auto (default):
        # every live_probe_every steps the share of dead waves (no sample with dL/dsigma != 0) of the last step
        # is read back asynchronously (no host sync: an event polled at the next steps), and the live backward
        # runs while the share exceeds live_on (back to the full one below live_off).
        self.live_bwd = {"0": False, "1": True}.get(os.environ.get("LONER_LIVE_BWD", "auto"), "auto")
        self.live_on, self.live_off, self.live_probe_every = 0.25, 0.15, 16
        self._live = self.live_bwd is True
        self._probe_ev, self._probe_ctr, self._probe_n = None, self.live_probe_every, 1
        self._probe_host = torch.zeros(1, dtype=torch.int64).pin_memory() if torch.cuda.is_available() else None
        # Joint pose + map (loner_amd.pose): with pose_grad on, the step also writes per ray [dL/d|d|, dL/dfar]
        # (d_ray, from the field kernel) and per sample dL/dpos01 (d_pos, the hash grid's input gradient,
        # before the table's Adam); ``poses`` (a pose.PoseWindow) then takes its Adam step after every
        # step_window step and rewrites the window's pose rows, which the next step's ray build reads
        self.pose_grad = False
        self.map_frozen = False
        self.poses = None
        self.d_ray = self.d_pos = None
        self._last_batch = None
        # Early ray termination: a sample behind enough opaque ones has float transmittance exactly 0 in the
        # compositing, so its weight is 0 and neither its sigma nor its encoding can change any output
        # (csrc/field.hip, LNR_ERT_T_MIN; 45 % of a trained C2 batch lies behind T = 0, tools/dead_bound.py).  The
        # forward then runs in phases of samples per ray (ert_bounds): each phase encodes and evaluates the rays still
        # alive and updates their transmittance, and a ray below 1e-50 skips the later phases.  Bitwise the step
        # without it (tests/test_gpu_live.py).  LONER_ERT: auto (default): the compositing counts where every ray
        # terminates (term_hist, lnr_loss_params.dev_term_hist), read back like the live backward's probe (no host
        # sync), and ert_plan picks the phases, or none, from the last steps' counts under a fitted cost model
        # (on the trained C2 field three cuts, on C4's forest, where few rays terminate,
        # none); 1: always, at the fixed cuts LONER_ERT_CUTS (fractions of n_samples, default 0.5,0.625,0.75); 0: never.
        self.ert = {"0": False, "1": True}.get(os.environ.get("LONER_ERT", "auto"), "auto")
        self.ert_cuts = [float(v) for v in os.environ.get("LONER_ERT_CUTS", "0.5,0.625,0.75").split(",") if v.strip()]
        # the phases' device state: the lists of rays still alive (two buffers, alternating), their counts, the
        # transmittance products and a scratch word per ray
        self.ert_lists = torch.zeros(2, max(n_rays, 1), dtype=torch.int32, device=dev)
        self.ert_counts = torch.zeros(2, dtype=torch.int32, device=dev)
        self.ert_T = torch.ones(n_rays, dtype=torch.float64, device=dev)
        self.ert_keep = torch.zeros(max(n_rays, 1), dtype=torch.int32, device=dev)
        self._ert_est = None  # auto: the plan's alive shares after each 64-sample boundary (the encode's grid hints)
        self._ert_last = None  # the phases of the last step (tests, tools)
        self._ert_plan = None  # auto: the phases in use, [0, c1, .., S], or None
        self._ert_next = None  # auto: (plan, alive shares) waiting for the next window (graph replay)
        nb = self.S // 64 + 1
        self.term_hist = (torch.zeros(TERM_HIST_SLOTS, nb, dtype=torch.int32, device=dev) if self.S % 64 == 0
                          else None)  # (slots spread the compositing's atomics; ert_probe sums them)
        pin = torch.cuda.is_available() and self.term_hist is not None
        self._term_host = torch.zeros(TERM_HIST_SLOTS, nb, dtype=torch.int32).pin_memory() if pin else None
        self._term_prev = [0] * (self.S // 64 + 1)
        self._term_ev, self._term_ctr = None, self.live_probe_every
        self._pp_bufs = [dict(rays=self.rays if i == 0 else torch.empty_like(self.rays),
                              dgt=self.depth_gt if i == 0 else torch.empty_like(self.depth_gt),
                              valid=self.ray_valid if i == 0 else torch.empty_like(self.ray_valid),
                              far=self.far_ref if i == 0 else torch.empty_like(self.far_ref),
                              z=self.z if i == 0 else torch.empty_like(self.z))
                         for i in range(2)]

    def ert_bounds(self):
        """The early-ray-termination phases [0, b1, ..., S] (whole 64-sample waves) of the coming step, or None:
        termination off (LONER_ERT=0, or auto with no plan that pays), or not applicable (n_samples not a multiple
        of 64 in {64 .. 512}, or fewer than two phases)."""
        S = self.S
        if not self.compact_denc or S % 64 or self.ert is False:
            return None
        if self.ert == "auto":
            return None if self._ert_plan is None else list(self._ert_plan)
        b = sorted({int(round(f * S / 64)) * 64 for f in self.ert_cuts if 0.0 < f < 1.0} - {0, S})
        return [0] + b + [S] if b else None

    def _mlp_adam(self, dsp, s):
        """Adam on the parameters outside the table (the MLP, and the padding tail), at st.adam_step."""
        st = self.state
        nm, nt = st.n_mlp, 2 * st.n_entries
        L.call("lnr_adam_step", st.params[:nm], st.shadow[:nm], st.grad[:nm], st.m[:nm], st.v[:nm], nm,
               st.adam_step, self.map_lr(), 0.9, 0.999, 1e-8, dsp, s)
        if st.n_padded > nm + nt:
            o = nm + nt
            L.call("lnr_adam_step", st.params[o:], st.shadow[o:], st.grad[o:], st.m[o:], st.v[o:], st.n_padded - o,
                   st.adam_step, self.map_lr(), 0.9, 0.999, 1e-8, dsp, s)

    def fuses_adam(self, N=None):
        """Whether the step runs the table's Adam inside the backward's accumulation (LONER_FUSED_ADAM: 1, 0, auto):
        one GPU (no exchange), the compact encoding gradient, and (auto) a batch of at most FUSED_ADAM_MAX_N samples
        or the live backward, whose unit accumulation takes the epilogue without spilling (the record-balanced one
        of a large full backward does not: k_bwd_accum<*, true>); C2 trained 0.949 -> 0.934 ms, C4 1.199 -> 1.182
        (the separate Adam's 237 MB of table traffic moves under the LDS-bound accumulation)."""
        N = self.N if N is None else N
        return self.allreduce is None and self.zero is None and self.compact_denc and (
            self.fused_adam is True or (self.fused_adam == "auto" and (N <= FUSED_ADAM_MAX_N or self._live)))

    def ert_alive_last(self):
        """The share of the last step's rays still alive after its last cut (early ray termination), or 1.0
        without phases (a host sync: tests and tools)."""
        b = self._ert_last
        if b is None or len(b) < 3:
            return 1.0
        return int(self.ert_counts[(len(b) - 3) % 2].item()) / max(self._r_last, 1)

    def _ert_key(self):
        b = self.ert_bounds()
        return None if b is None else tuple(b)

    def ert_probe(self):
        """LONER_ERT=auto: re-plan the phases from the termination counts the steps since the last probe added to
        term_hist (read back behind an event, no host sync; the first probe after the first step, then every
        live_probe_every steps)."""
        if self.ert != "auto" or self._term_host is None:
            return
        ev = self._term_ev
        if ev is not None and ev.query():
            cur = [int(v) & 0xFFFFFFFF for v in self._term_host.long().sum(0).tolist()]
            d = [(c - p) & 0xFFFFFFFF for c, p in zip(cur, self._term_prev)]  # (the counters wrap at 2^32)
            self._term_prev = cur
            self._term_ev = None
            if sum(d) > 0:
                # a window replaying graphs keeps its plan: a new plan would cost an eager step and a capture
                # mid-window (~2 ms), so it takes effect with the next window's captures, which are made anyway
                # (no margin for those: the cheapest plan of the latest counts)
                defer = self._ert_est is not None and self._graph_window is not None
                plan = ert_plan(d, self.S, self._r_last * self.S, self._ert_plan,
                                margin=0.0 if defer else ERT_MARGIN)
                if plan != self._ert_plan or self._ert_est is None:
                    # the alive shares behind the encode's grid hints: refreshed with the plan only (the graphs,
                    # captured per plan, hold the hints of their capture)
                    nxt = (plan, [float(v) for v in ert_alive(d, self.S)])
                    if defer:
                        self._ert_next = nxt
                    else:
                        self._ert_plan, self._ert_est = nxt
                        self._ert_next = None
                else:
                    self._ert_next = None  # the latest counts confirm the plan in use
        self._term_ctr += 1
        if self._term_ev is None and self._term_ctr >= self.live_probe_every:
            self._term_ctr = 0
            self._term_host.copy_(self.term_hist, non_blocking=True)
            self._term_ev = torch.cuda.Event()
            self._term_ev.record()

    def map_lr(self):
        """The map's Adam learning rate this step: lrate_sigma_mlp x the ExponentialLR factor, or 0 while the
        map is frozen (``map_frozen``: pose tracking, optimizer.py:232,255-257; Adam with a zero step size
        leaves every parameter bit for bit as it is)."""
        return 0.0 if self.map_frozen else self.cfg.lr * self.lr_factor

    def set_poses(self, poses):
        """Optimise the window's poses with the map (``poses``: a loner_amd.pose.PoseWindow), or stop (None).
        The pose gradient's buffers are allocated on first use."""
        self.poses = poses
        self.pose_grad = poses is not None
        if self.pose_grad and self.d_ray is None:
            dev = self.state.device
            self.d_ray = torch.zeros(self.n_rays, 2, dtype=torch.float32, device=dev)
            self.d_pos = torch.zeros(self.N, 3, dtype=torch.float32, device=dev)
        self.drop_prefetch()  # a prefetched build read the poses before this step's update

    def loss_params(self, global_step, iteration_idx, scale, far_ref, n_rays_global, dev_far_ref=None):
        lc = self.cfg.loss
        lp = L.LossParams()
        lp.kind = L.LOSS_KINDS[lc.loss_selection]
        lp.scale = float(scale)
        lp.los_lambda = float(lc.los_lambda_at(global_step))
        lp.depthloss_lambda = lc.depthloss_lambda
        lp.min_depth_eps = lc.min_depth_eps
        lp.min_js = lc.min_js_score
        lp.max_js = lc.max_js_score
        lp.js_alpha = lc.js_alpha
        lp.los_eps = float(lc.los_eps_at(iteration_idx))
        lp.far_ref = 0.0 if far_ref is None else float(far_ref)
        lp.inv_n_opaque = 0.0
        lp.inv_rs = 1.0 / float(n_rays_global * self.S)
        lp.dev_n_opaque = self.n_opaque.data_ptr()
        lp.dev_far_ref = None if dev_far_ref is None else dev_far_ref.data_ptr()
        lp.dev_status = self.status.data_ptr()
        # lnr_field_train stores the MLP gradient (no zeroing launch) and finalizes the loss scalars
        # into loss_out in its last launch (no lnr_loss_finalize launch)
        lp.dev_loss_out = self.loss_out.data_ptr()
        lp.flags = L.LP_DW_OVERWRITE
        return lp

    def check_status(self, clear=True):
        """Read the device status word (one host sync; call it as often as the caller wants, e.g. once
        per window).  Raises like the reference's per-step ``assert not torch.isnan(loss), "NaN Loss
        Encountered"`` (optimizer.py:854) and warns once, like DecoupledNeRF (nerf_tcnn.py:74-78),
        when a non-finite sigma was clipped.  Returns the bits."""
        bits = int(self.status.item())
        if clear:
            self.status.zero_()
        if bits & L.STATUS_SIGMA_CLIPPED and not self._warned_clip:
            self._warned_clip = True
            warnings.warn("Clipping infinite outputs. Will not warn about this again (but it will happen again)")
        if bits & L.STATUS_NAN_LOSS:
            raise RuntimeError("NaN Loss Encountered")
        return bits

    def _ar_range(self, l0, l1):
        """[a0, a1) of level range [l0, l1) in the flat parameter buffer (range 0 also holds the MLP)."""
        st = self.state
        a0 = 0 if l0 == 0 else st.n_mlp + 2 * int(st.desc.offset[l0])
        return a0, st.n_mlp + 2 * int(st.desc.offset[l1])

    def sync_master(self):
        """Sharded optimiser: all-gather the fp32 master (and the Adam moments) chunks so every rank holds
        the whole current state (e.g. before a checkpoint).  A no-op otherwise."""
        self.finish()
        if self.zero is None or self.zero[1] == 1 or self.all_gather is None:
            return
        st, (zr, zw) = self.state, self.zero
        for a0, a1, c in self.zero_chunks:
            for buf in (st.params, st.m, st.v):
                self.all_gather(buf[a0:a1], buf[a0 + zr * c:a0 + (zr + 1) * c])

    def _allreduce_async(self, t):
        """``allreduce(t, async_op=True)`` when the hook supports it (torch.distributed's
        all_reduce does: the returned work's wait() makes the current stream wait), else a
        blocking call."""
        try:
            return self.allreduce(t, async_op=True)
        except TypeError:
            self.allreduce(t)
            return None

    @staticmethod
    def _mark(prof, stage):
        """Record a HIP event on the current stream (the stream every kernel here is launched on)."""
        if prof is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            prof.setdefault(stage, []).append(ev)

    def step(self, rays, depth_gt, global_step, iteration_idx=0, scale=1.0, far_ref=None, n_rays_global=None,
             u_jitter=None, u_pdf=None, noise=None, update_ogm=None, prof=None, presampled=False, dev_step=None,
             fork_count=True):
        """rays (R,13) fp32, depth_gt (R,) fp32 normalised, both on this GPU, R <= the engine's
        capacity.  Returns the device loss buffer [loss, mean_eps, depth_term, los_term, opacity_term,
        n_opaque] (no host sync).  ``far_ref``: the far bound of global ray 0, a float or a 1-element
        device tensor.  ``prof``: optional dict collecting (begin, end) HIP event pairs per stage.
        ``dev_step``: a device ``lnr_step_scalars`` holding this step's key, loss scalars and Adam
        coefficients, read by the kernels instead of their host arguments (the graph-captured step)."""
        st = self.state
        cfg = self.cfg
        R, S, N = rays.shape[0], self.S, self.N  # N: the level stride of enc / d_enc (capacity)
        assert rays.shape == (R, 13) and depth_gt.shape == (R,) and R <= self.n_rays, (rays.shape, self.n_rays)
        s = L.stream(st.device)
        key = L.step_key(self.seed, global_step)
        if far_ref is None:
            raise ValueError("far_ref (far bound of global ray 0) is required; optimizer.py:724")
        dev_far = far_ref if isinstance(far_ref, torch.Tensor) else None
        far_h = None if dev_far is not None else float(far_ref)
        n_glob = R if n_rays_global is None else n_rays_global
        m = self._mark
        # 1. opaque count (global): local count + all-reduce, on the side stream; the count is first
        # needed by the field kernel, so both overlap sampling + encode
        main = torch.cuda.current_stream(st.device)
        pending = None
        if fork_count or self.allreduce is not None:
            self._fork.record(main)
            with torch.cuda.stream(self._side):
                self._side.wait_event(self._fork)
                L.call("lnr_count_opaque", depth_gt, R, 0.0 if far_h is None else far_h, dev_far, self.n_opaque,
                       L.stream(st.device))
                pending = self._allreduce_async(self.n_opaque) if self.allreduce is not None else None
                self._join.record(self._side)
        else:  # (a captured single-stream step: the count inline, one stream in the graph)
            L.call("lnr_count_opaque", depth_gt, R, 0.0 if far_h is None else far_h, dev_far, self.n_opaque, s)
        lp = self.loss_params(global_step, iteration_idx, scale, far_h, n_glob, dev_far)
        dsp = None if dev_step is None else dev_step.data_ptr()
        lp.dev_step = dsp
        lp.dev_d_ray = self.d_ray.data_ptr() if self.pose_grad else None
        # (counted under fixed phases too, for the tools' alive shares: no measurable cost, C2 0.903 ms either way)
        lp.dev_term_hist = self.term_hist.data_ptr() if self.ert is not False and self.term_hist is not None else None
        self._dev_step = dsp
        # 2. sampling (``presampled``: step_window's pipeline already drew self.z for these rays); the previous
        # step's data-parallel OGM update lands first (the sampler reads the grid)
        self._apply_pending_ogm()
        m(prof, "sample")
        if presampled:
            pass
        elif cfg.sampler == "OGM":
            L.call("lnr_sample_ogm", rays, R, S, st.occ, cfg.occ_res, cfg.perturb, u_jitter, u_pdf, key,
                   self.ray_offset, self.z, dsp, s)
        else:
            L.call("lnr_sample_uniform", rays, R, S, cfg.perturb, u_jitter, key, self.ray_offset, self.z, dsp, s)
        m(prof, "sample")
        # 3. encode (+ backward record histogram); it reads the fp16 shadow, which the previous step's
        # sharded-optimiser all-gathers may still be writing
        self.finish()
        m(prof, "encode")
        # the backward's record histogram, counted from the forward's corners, for the full backward (the live one
        # counts its live records itself)
        fwd_hist = self.count_in_forward and not self._live
        ert = self.ert_bounds()
        self._ert_last = ert
        if ert is not None:
            # early ray termination (see __init__): phase by phase, the encode and sigma of the rays still alive
            # (the list phase q - 1 left; every ray in phase 0; a ray that terminates gets sigma 0 at its later samples)
            lp.flags |= L.LP_SIGMA_READY
            for q in range(len(ert) - 1):
                lo, hi = ert[q], ert[q + 1]
                hist = q == 0 and fwd_hist
                lin = None if q == 0 else self.ert_lists[(q - 1) % 2]
                cin = None if q == 0 else self.ert_counts[(q - 1) % 2:(q - 1) % 2 + 1]
                est = self._ert_est
                expect = 0 if (q == 0 or est is None) else int(est[lo // 64] * R) + 64
                L.call("lnr_hashgrid_fwd_rays_phase", L.ctypes.byref(st.desc), rays, self.z, R, S, st.table_f16,
                       self.enc, N, self.bwd_ws if hist else None, self.bwd_ws_bytes if hist else 0, lin, cin,
                       expect, lo, hi, s)
                m(prof, "sigma_phase")
                L.call("lnr_field_sigma_phase", st.mlp_f16, self.enc, N, rays, self.z, R, S, lo, hi,
                       cfg.raw_noise_std, noise, key, self.ray_offset, L.ctypes.byref(lp), self.ws, lin, cin,
                       self.ert_lists[q % 2], self.ert_counts[q % 2:q % 2 + 1], self.ert_T, self.ert_keep, s)
                m(prof, "sigma_phase")
        elif fwd_hist:
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rays, self.z, R, S, st.table_f16, self.enc, N,
                   self.bwd_ws, self.bwd_ws_bytes, s)
        else:
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rays, self.z, R, S, st.table_f16, self.enc, N,
                   None, 0, s)
        m(prof, "encode")
        # 4. fused field + loss + backward through compositing and MLP (stores the MLP gradient, and the
        # loss scalars into loss_out)
        if fork_count or self.allreduce is not None:
            main.wait_event(self._join)
        if pending is not None:
            pending.wait()  # orders the current stream after the collective (no host sync)
        flags = (L.BWD_COUNTS_READY if fwd_hist else 0) | L.BWD_LEVEL_MAX_READY | (
            L.BWD_LIVE if self._live else 0)
        split = (self.split_bwd and self._live and self.compact_denc and prof is None and self.allreduce is None
                 and self.zero is None and S in (64, 128, 256, 512))
        mlp_adam_done = False

        def field_train(extra):
            lp.flags |= extra
            L.call("lnr_field_train", st.mlp_f16, self.enc, N, rays, self.z, depth_gt, R, S, cfg.raw_noise_std, noise,
                   key, self.ray_offset, L.ctypes.byref(lp), self.d_enc, st.grad_mlp, self.ws, self.stats, self.depth,
                   self.opacity, None, self.level_max_ptr, self.d_jac if self.compact_denc else None, s)
            lp.flags &= ~extra

        m(prof, "field")
        if split:
            # compositing (dL/dsigma), then the backward's preparation on the side stream beside the MLP backward
            field_train(L.LP_FORWARD_ONLY)
            self._bfork.record(main)
            with torch.cuda.stream(self._bside):
                self._bside.wait_event(self._bfork)
                L.call("lnr_hashgrid_bwd_rays_jac", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_jac,
                       self.d_sigma(R), N, st.grad_table, None, None, self.bwd_ws, self.bwd_ws_bytes,
                       flags | L.BWD_PREPARE_ONLY, L.stream(st.device))
                self._bjoin.record(self._bside)
            field_train(L.LP_BACKWARD_ONLY)
            if self.fuses_adam(N):
                # the MLP's Adam (its gradient is complete) while the side stream still prepares the backward
                st.adam_step += 1
                self._mlp_adam(dsp, s)
                mlp_adam_done = True
            main.wait_event(self._bjoin)
            flags |= L.BWD_PREPARED
        else:
            field_train(0)
        m(prof, "field")
        self._r_last = R
        if self.pose_grad:
            # 4b. the poses' share: dL/dpos01 per sample (tcnn's input gradient) from the table the forward read,
            # before the table's Adam (below) changes it
            m(prof, "pose_grad")
            if self.compact_denc:
                L.call("lnr_hashgrid_bwd_rays_jac", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_jac,
                       self.d_sigma(R), N, None, st.table_f16, self.d_pos, None, 0, 0, s)
            else:
                L.call("lnr_hashgrid_bwd_rays", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_enc, N, None,
                       st.table_f16, self.d_pos, None, 0, 0, s)
            m(prof, "pose_grad")
        # 5. hash-grid backward
        m(prof, "grid_bwd")
        if self.zero is not None:
            return self._step_zero(rays, depth_gt, R, S, N, flags, s, scale, update_ogm, global_step, prof)
        if self.fuses_adam(N):
            # 5 + 7. the table's Adam inside the backward (lnr_hashgrid_bwd_rays_jac_adam: each entry's
            # gradient updates its parameter where the accumulation finishes it, bitwise lnr_adam_step's
            # result), then Adam on the MLP's parameters alone
            if not mlp_adam_done:
                st.adam_step += 1
            st.grad_table_current = False
            nm, nt = st.n_mlp, 2 * st.n_entries
            epi = L.AdamEpilogue(L.ptr(st.params[nm:nm + nt]), L.ptr(st.shadow[nm:nm + nt]), L.ptr(st.m[nm:nm + nt]),
                                 L.ptr(st.v[nm:nm + nt]), st.adam_step, self.map_lr(), 0.9, 0.999, 1e-8, dsp)
            L.call("lnr_hashgrid_bwd_rays_jac_adam", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_jac,
                   self.d_sigma(R), N, L.ctypes.byref(epi), self.bwd_ws, self.bwd_ws_bytes, flags, s)
            m(prof, "grid_bwd")
            m(prof, "adam")
            if not mlp_adam_done:
                self._mlp_adam(dsp, s)
            m(prof, "adam")
            if update_ogm is None:
                update_ogm = (global_step % cfg.n_iters_acc == 0)
            if update_ogm:
                m(prof, "ogm")
                self.ogm_update(rays, depth_gt, scale)
                m(prof, "ogm")
            return self.loss_out
        if self.allreduce is None:
            self._grid_bwd(rays, R, S, N, flags, s)
            m(prof, "grid_bwd")
        else:
            # 6. data-parallel gradient exchange, bucketed by level range: each range's slice of the
            # gradient is all-reduced (async) while the next range accumulates; the MLP gradient
            # travels with the last range
            self._grid_bwd(rays, R, S, N, flags | L.BWD_NO_ACCUM, s)
            pending = []
            for l0, l1 in self.ar_groups:
                L.call("lnr_hashgrid_bwd_accum_flags", L.ctypes.byref(st.desc), R * S, self.bwd_ws, self.bwd_ws_bytes,
                       l0, l1, st.grad_table, flags & L.BWD_LIVE, s)
                a0, a1 = self._ar_range(l0, l1)
                pending.append(self._allreduce_async(st.grad[a0:a1]))
            m(prof, "grid_bwd")
            m(prof, "allreduce")
            for w in pending:
                if w is not None:
                    w.wait()
            m(prof, "allreduce")
        # 7. Adam (+ fp16 shadow)
        st.adam_step += 1
        m(prof, "adam")
        L.call("lnr_adam_step", st.params, st.shadow, st.grad, st.m, st.v, st.n_padded, st.adam_step,
               self.map_lr(), 0.9, 0.999, 1e-8, dsp, s)
        m(prof, "adam")
        # 8. OGM every N_iters_acc global steps (optimizer.py:466-469)
        if update_ogm is None:
            update_ogm = (global_step % cfg.n_iters_acc == 0)
        if update_ogm:
            m(prof, "ogm")
            self.ogm_update(rays, depth_gt, scale)
            m(prof, "ogm")
        return self.loss_out

    def _step_zero(self, rays, depth_gt, R, S, N, flags, s, scale, update_ogm, global_step, prof):
        """The step's tail with the sharded optimiser (see __init__), pipelined per level range: each range
        is accumulated and its gradient slice reduce-scattered (asynchronous: the next range accumulates
        meanwhile); then, range by range as its reduce-scatter lands, Adam on this rank's chunk of it and
        the all-gather of that chunk's fp16 shadow (asynchronous).  Nothing waits for the all-gathers here:
        the next reader of the shadow (the next step's encode, after its ray build and sampling, or
        finish()) does, so the gather overlaps the next step's head.  Exposed per step: the last range's
        reduce-scatter and its Adam (the cut: AR_CUT_DEFAULT)."""
        st, cfg, m = self.state, self.cfg, self._mark
        zr, zw = self.zero
        comm = self.allreduce is not None and zw > 1
        rs = [None] * len(self.zero_chunks)
        if comm:
            self._grid_bwd(rays, R, S, N, flags | L.BWD_NO_ACCUM, s)
            for i, ((l0, l1), (a0, a1, c), out) in enumerate(zip(self.ar_groups, self.zero_chunks, self.zero_grad)):
                L.call("lnr_hashgrid_bwd_accum_flags", L.ctypes.byref(st.desc), R * S, self.bwd_ws, self.bwd_ws_bytes,
                       l0, l1, st.grad_table, flags & L.BWD_LIVE, s)
                rs[i] = self.reduce_scatter(out, st.grad[a0:a1], async_op=True)
            m(prof, "grid_bwd")
        else:  # one process: this rank's share of the work only (no exchange)
            self._grid_bwd(rays, R, S, N, flags, s)
            m(prof, "grid_bwd")
        st.adam_step += 1
        m(prof, "adam")
        lr = self.map_lr()
        if not comm:
            # this rank's chunk of every level range, one launch (lnr_adam_step_ranges)
            rng = (L.AdamRange * len(self.zero_chunks))()
            for i, (a0, a1, c) in enumerate(self.zero_chunks):
                o = a0 + zr * c
                rng[i] = L.AdamRange(L.ptr(st.params[o:o + c]), L.ptr(st.shadow[o:o + c]), L.ptr(st.grad[o:o + c]),
                                     L.ptr(st.m[o:o + c]), L.ptr(st.v[o:o + c]), c)
            L.call("lnr_adam_step_ranges", rng, len(self.zero_chunks), st.adam_step, lr, 0.9, 0.999, 1e-8,
                   self._dev_step, s)
        else:
            pend = []
            for i, ((a0, a1, c), g) in enumerate(zip(self.zero_chunks, self.zero_grad)):
                if rs[i] is not None:
                    rs[i].wait()  # orders the current stream after this range's reduce-scatter
                o = a0 + zr * c
                L.call("lnr_adam_step", st.params[o:o + c], st.shadow[o:o + c], g, st.m[o:o + c], st.v[o:o + c], c,
                       st.adam_step, lr, 0.9, 0.999, 1e-8, self._dev_step, s)
                pend.append(self.all_gather(st.shadow[a0:a1], st.shadow[o:o + c], async_op=True))
            self._pending_shadow = [w for w in pend if w is not None]
            if prof is not None:
                self.finish()  # a profiled step keeps its stages apart
        m(prof, "adam")
        if update_ogm is None:
            update_ogm = (global_step % cfg.n_iters_acc == 0)
        if update_ogm:
            m(prof, "ogm")
            self.ogm_update(rays, depth_gt, scale)
            m(prof, "ogm")
        return self.loss_out

    def live_probe(self, n_rays=None):
        """LONER_LIVE_BWD=auto: pick the backward for the coming steps from the share of dead 64-sample waves
        (see __init__).  Called after every step by step_window; a probe is a count of the last step's waves
        holding a non-zero dL/dsigma, copied to pinned host memory behind an event, read when the event has
        completed.  Also runs the early-ray-termination probe (ert_probe)."""
        self.ert_probe()
        if self.live_bwd != "auto":
            return
        ev = self._probe_ev
        if ev is not None and ev.query():
            dead = 1.0 - float(self._probe_host[0]) / self._probe_n
            self._live = dead > (self.live_off if self._live else self.live_on)
            self._probe_ev = None
        self._probe_ctr += 1
        if ev is None and self._probe_ctr >= self.live_probe_every and self._probe_host is not None:
            self._probe_ctr = 0
            r = self._r_last if n_rays is None else n_rays
            nw = r * self.S // 64
            live_waves = torch.count_nonzero(self.d_sigma(r)[:64 * nw].view(nw, 64).ne(0).any(1))
            self._probe_host.copy_(live_waves.view(1), non_blocking=True)
            self._probe_n = max(nw, 1)
            self._probe_ev = torch.cuda.Event()
            self._probe_ev.record()

    def finish(self):
        """Order the current stream after the sharded optimiser's pending shadow all-gathers (the shadow is
        then whole again).  step() calls it before its encode; call it before reading the fp16 parameters
        elsewhere (checkpoints, evaluation on the same FieldState).  A no-op without pending gathers."""
        self._apply_pending_ogm()
        pend, self._pending_shadow = self._pending_shadow, []
        for w in pend:
            w.wait()

    def d_sigma(self, n_rays=None):
        """dL/dsigma (n_rays * S) of the last step: lnr_field_train leaves it in its workspace after the dW
        slabs, whose count follows the call's ray count."""
        r = self._r_last if n_rays is None else n_rays
        off = int(L.lib().lnr_dw_workspace_words(r))
        return self.ws[off:off + r * self.S]

    def denc_f32(self):
        """The last step's encoding gradient as (L, N, 2) fp32 (tests and tools; the step itself keeps
        the compact form: d_sigma * J, computed exactly so in the backward)."""
        if not self.compact_denc:
            return self.d_enc
        nl, n = self.cfg.n_levels, self._r_last * self.S
        ds = self.d_sigma().view(1, n, 1)
        # (J is not written where a 32-sample pair's dL/dsigma are all 0: d_enc is 0 there, include/loner_amd.h)
        return torch.where(ds == 0, 0.0, self.d_jac.view(torch.float16).view(nl, self.N, 2)[:, :n].float() * ds)

    def _grid_bwd(self, rays, R, S, N, flags, s):
        st = self.state
        st.grad_table_current = True
        if self.compact_denc:
            L.call("lnr_hashgrid_bwd_rays_jac", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_jac,
                   self.d_sigma(R), N, st.grad_table, None, None, self.bwd_ws, self.bwd_ws_bytes, flags, s)
        else:
            L.call("lnr_hashgrid_bwd_rays", L.ctypes.byref(st.desc), rays, self.z, R, S, self.d_enc, N, st.grad_table,
                   None, None, self.bwd_ws, self.bwd_ws_bytes, flags, s)

    def ogm_update(self, rays, depth_gt, scale):
        """Optimizer._step_occupancy_grid (optimizer.py:897-908).  Data-parallel: the grid gradient
        is all-reduced before the SGD step so every replica applies the global-batch update; the all-reduce
        is asynchronous and the SGD step waits for it at the grid's next reader (``_apply_pending_ogm``)."""
        st = self.state
        s = L.stream(st.device)
        if self.allreduce is None:
            L.call("lnr_ogm_update", (rays), (self.z), (depth_gt), rays.shape[0], self.S, float(scale),
                   self.cfg.occ_lr, (st.occ), (st.occ_ws), st.occ_ws.numel(), self.cfg.occ_res, s)
            return
        L.call("lnr_ogm_grad", (rays), (self.z), (depth_gt), rays.shape[0], self.S, float(scale),
               (st.occ_ws), st.occ_ws.numel(), self.cfg.occ_res, s)
        g = st.occ_ws[:st.occ.numel()]
        # asynchronous: nothing on this step's stream waits for it; the SGD step is enqueued (after a wait on
        # the collective) right before the grid's next reader (_apply_pending_ogm)
        self._pending_ogm = (self._allreduce_async(g), g)

    def _apply_pending_ogm(self):
        """Enqueue the data-parallel OGM step's SGD update once its gradient all-reduce is waited for (a
        no-op without one pending)."""
        p, self._pending_ogm = self._pending_ogm, None
        if p is None:
            return
        w, g = p
        if w is not None:
            w.wait()  # orders the current stream after the collective (no host sync)
        L.call("lnr_sgd_step", self.state.occ, g, self.state.occ.numel(), self.cfg.occ_lr, L.stream(self.state.device))

    def step_window(self, window, global_step, iteration_idx=0, n_rays_global=None, prof=None, n_slots=None, **kw):
        """One optimiser step whose rays are selected and built on the device from a resident
        ``loner_amd.rays.RayWindow`` (optimizer.py:363-424 + the step above).  This rank builds the
        window's slots [ray_offset, ray_offset + n_slots) (n_slots <= capacity, default the
        capacity).  When the window can produce invalid rays (``window.all_valid`` False) they are
        dropped as the reference drops them, which needs the batch size on the host: one
        synchronisation, only on such windows."""
        n = self.n_rays if n_slots is None else int(n_slots)
        if not 0 <= n <= self.n_rays or self.ray_offset + n > window.n_slots:
            raise ValueError(f"slots [{self.ray_offset}, {self.ray_offset + n}) outside the window "
                             f"({window.n_slots}) or the engine capacity ({self.n_rays})")
        if self.poses is not None and self.poses.window is not window:
            raise ValueError("step_window: the engine's PoseWindow belongs to another window (set_poses)")
        out = self._step_window_any(window, global_step, iteration_idx, n, n_rays_global, prof, kw)
        if self.poses is not None:
            # joint pose + map: the poses' Adam step on this step's gradient; the next build reads the new poses
            m = self._mark
            m(prof, "pose_adam")
            rays, slots = self._last_batch
            self.poses.step(self, rays, slots, self.lr_factor)  # (slots None: the engine's [ray_offset, + n))
            m(prof, "pose_adam")
        return out

    def _step_window_any(self, window, global_step, iteration_idx, n, n_rays_global, prof, kw):
        m = self._mark
        if window.all_valid and (self.poses is None or self.poses.stay_valid):
            out = self._step_window_pipelined(window, global_step, iteration_idx, n, n_rays_global, prof, kw)
            if self.poses is not None:
                self._last_batch = (self.rays[:n], None)
            return out
        # Windows with rays the 1 m filter drops: the batch size must reach the host (one sync per step).
        # The build and compaction of step k + 1 run on a side stream while step k runs, so that sync
        # never waits for the main stream: the host stays a step ahead of the GPU (double-buffered).
        main = torch.cuda.current_stream(self.state.device)
        want = (global_step, n, self.ray_offset, n_rays_global)
        pf, self._pf = self._pf, None
        if pf is not None:
            # a prefetch is consumed or discarded only after the main stream waits for it, so the
            # window it read (kept alive by pf["window"] until now) is free for reuse afterwards
            main.wait_event(pf["done"])
        if pf is None or pf["window"] is not window or pf["want"] != want:
            m(prof, "rays")
            pf = self._build_compact(window, global_step, n, n_rays_global, self._pf_parity, main)
            m(prof, "rays")
        self._pf_parity = pf["parity"]
        self._pf_fork.record(main)  # the other buffer is free once everything enqueued so far is done
        out = self.step(pf["rays"], pf["dgt"], global_step, iteration_idx, scale=window.scale, far_ref=pf["far"],
                        n_rays_global=pf["n_glob"], prof=prof, **kw)
        self.live_probe(pf["rays"].shape[0])
        if self.poses is not None:
            self._last_batch = (pf["rays"], pf["slots"])
            return out  # (no prefetch: the next build must read the poses this step's pose update writes)
        if self.prefetch:
            nxt = None if n_rays_global is None else n_rays_global
            with torch.cuda.stream(self._pf_stream):
                self._pf_stream.wait_event(self._pf_fork)
                self._pf = self._build_compact(window, global_step + 1, n, nxt, 1 - self._pf_parity, self._pf_stream)
        return out

    def _step_window_pipelined(self, window, global_step, iteration_idx, n, n_rays_global, prof, kw):
        """step_window for windows with no invalid rays (fixed batch size, no host sync), with step
        k + 1's build + sampling prefetched (``pipeline``)."""
        if (self.use_graph and prof is None and self.allreduce is None and not
                any(k in kw for k in ("u_jitter", "u_pdf", "noise", "presampled"))):
            return self._step_window_graph(window, global_step, iteration_idx, n, n_rays_global, kw)
        m = self._mark
        main = torch.cuda.current_stream(self.state.device)
        want = (global_step, n, self.ray_offset)
        pp, self._pp = self._pp, None
        if pp is not None:
            # consumed or discarded, the prefetch is waited for first: the main stream's later work
            # (and the caching allocator's reuse of the window it read, which pp["window"] kept alive
            # until here) is ordered after its side-stream reads
            main.wait_event(pp["done"])
        if pp is not None and pp["window"] is window and pp["want"] == want:
            parity, presampled = pp["parity"], pp["sampled"]
            b = self._pp_bufs[parity]
        else:
            parity, presampled = self._pp_parity, False
            b = self._pp_bufs[parity]
            m(prof, "rays")
            window.build(L.step_key(self.seed, global_step), self.ray_offset, n, b["rays"][:n], b["dgt"][:n],
                         b["valid"][:n], None, b["far"])
            m(prof, "rays")
        self._pp_parity = parity
        # (the buffers of the step in flight: rays, depth_gt, ray_valid, far_ref and z as step() uses them)
        self.z, self.rays, self.depth_gt, self.ray_valid, self.far_ref = b["z"], b["rays"], b["dgt"], b["valid"], b["far"]
        # the previous step's data-parallel OGM update (its SGD step, pending until the grid's next reader) lands
        # before the fork: the prefetch below samples the grid on the side stream after waiting on this fork only
        self._apply_pending_ogm()
        self._pp_fork.record(main)  # the other buffers are free once everything enqueued so far is done
        out = self.step(b["rays"][:n], b["dgt"][:n], global_step, iteration_idx, scale=window.scale, far_ref=b["far"],
                        n_rays_global=window.n_slots if n_rays_global is None else n_rays_global, prof=prof,
                        presampled=presampled, **kw)
        self.live_probe(n)
        if not self.pipeline or prof is not None or "u_jitter" in kw or "u_pdf" in kw or self.poses is not None:
            return out  # (a profiled step keeps its stages apart; a pose step's update precedes the next build)
        cfg = self.cfg
        ogm_now = kw.get("update_ogm")
        if ogm_now is None:
            ogm_now = global_step % cfg.n_iters_acc == 0
        q = 1 - parity
        bq = self._pp_bufs[q]
        key = L.step_key(self.seed, global_step + 1)
        sample = cfg.sampler != "OGM" or not ogm_now  # the OGM sampler reads the grid step k may update
        with torch.cuda.stream(self._pp_stream):
            self._pp_stream.wait_event(self._pp_fork)
            window.build(key, self.ray_offset, n, bq["rays"][:n], bq["dgt"][:n], bq["valid"][:n], None, bq["far"])
            if sample:
                s = L.stream(self.state.device)
                if cfg.sampler == "OGM":
                    L.call("lnr_sample_ogm", bq["rays"][:n], n, self.S, self.state.occ, cfg.occ_res, cfg.perturb, None,
                           None, key, self.ray_offset, bq["z"], None, s)
                else:
                    L.call("lnr_sample_uniform", bq["rays"][:n], n, self.S, cfg.perturb, None, key, self.ray_offset,
                           bq["z"], None, s)
            done = torch.cuda.Event()
            done.record(self._pp_stream)
        self._pp = dict(window=window, want=(global_step + 1, n, self.ray_offset), parity=q, sampled=sample, done=done)
        return out

    def drop_prefetch(self):
        """Discard a pending prefetch (the main stream waits for its side-stream work, then the window it
        read is released).  step_window does this itself when the next call does not match."""
        main = torch.cuda.current_stream(self.state.device)
        for pend in (self._pp, self._pf):
            if pend is not None:
                main.wait_event(pend["done"])
        self._pp = self._pf = None
        self.finish()

    def release(self):
        """End of a window: drop_prefetch(), and the HIP graphs captured for this window with the window
        itself (their captured pointers keep its device tensors alive), so two windows' resident data never
        coexist.  Optimizer calls it when a window's iterations are done."""
        self.drop_prefetch()
        self._graphs.clear()
        self._graph_window = None
        self._ert_adopt()

    def _ert_adopt(self):
        """A window boundary: the plan ert_probe deferred while graphs replayed takes effect."""
        if self._ert_next is not None:
            self._ert_plan, self._ert_est = self._ert_next
            self._ert_next = None

    def step_scalars(self, global_step, iteration_idx=0, adam_step=None):
        """The host ``lnr_step_scalars`` of a step: the values the eager step passes as kernel arguments
        (the same host arithmetic), for a captured step to read from device memory."""
        st, cfg = self.state, self.cfg
        sc = L.StepScalars()
        sc.key = L.step_key(self.seed, global_step)
        sc.los_lambda = float(cfg.loss.los_lambda_at(global_step))
        sc.los_eps = float(cfg.loss.los_eps_at(iteration_idx))
        t = st.adam_step + 1 if adam_step is None else adam_step
        a, b = L.ctypes.c_float(), L.ctypes.c_float()
        L.check(L.lib().lnr_adam_coefficients(t, self.map_lr(), 0.9, 0.999, L.ctypes.byref(a),
                                              L.ctypes.byref(b)), "lnr_adam_coefficients")
        sc.adam_step_size, sc.adam_bc2_sqrt = a.value, b.value
        return sc

    def _step_window_graph(self, window, global_step, iteration_idx, n, n_rays_global, kw):
        """step_window as a replayed HIP graph (see __init__): the whole step, ray build included, on one stream.
        Graphs are captured per (OGM step or not, batch, backward) and per window: the first step of each runs
        eagerly with the device scalars (every kernel loaded; the step's own result) and is then captured without
        executing; later steps set their scalars (one small launch) and replay.  Bitwise the eager path
        (tests/test_gpu_rays.py::test_graph_replay_equals_eager).  (The next step's build + sampling as a forked
        branch of the graph measured slower than the single-stream graph at every fork point, round 5: DESIGN.md
        section 4d; removed in round 6, commit history before e32a0b7.)"""
        st, cfg = self.state, self.cfg
        if self._pp is not None or self._pf is not None:
            self.drop_prefetch()
        self.finish()
        ogm = kw.get("update_ogm")
        if ogm is None:
            ogm = global_step % cfg.n_iters_acc == 0
        ogm = bool(ogm)
        n_glob = window.n_slots if n_rays_global is None else n_rays_global
        if self._graph_window is not window:  # a new window: its tensors back the captured pointers
            self._graphs.clear()
            self._graph_window = window
            self._ert_adopt()
        p = self._pp_parity
        gkey = (p, ogm, n, self.ray_offset, n_glob, self.zero, self._live, self.pose_grad, self._ert_key())
        s = L.stream(st.device)
        sc = (L.StepScalars * 1)()
        sc[0] = self.step_scalars(global_step, iteration_idx)
        L.call("lnr_step_scalars_set", sc, 1, self._dev_steps, s)
        b = self._pp_bufs[p]
        self.z, self.rays, self.depth_gt, self.ray_valid, self.far_ref = b["z"], b["rays"], b["dgt"], b["valid"], b["far"]

        def body():
            window.build(sc[0].key, self.ray_offset, n, b["rays"][:n], b["dgt"][:n], b["valid"][:n], None, b["far"],
                         dev_step=self.dev_step)
            return self.step(b["rays"][:n], b["dgt"][:n], global_step, iteration_idx, scale=window.scale,
                             far_ref=b["far"], n_rays_global=n_glob, update_ogm=ogm, dev_step=self.dev_step,
                             fork_count=False)

        g = self._graphs.get(gkey)
        if g is not None:
            g.replay()
            st.adam_step += 1
            self._r_last = n
            self.live_probe(n)
            return self.loss_out
        out = body()  # this step, eagerly
        saved = st.adam_step
        g = torch.cuda.CUDAGraph()
        cs = self._capture_stream
        cs.wait_stream(torch.cuda.current_stream(st.device))
        with torch.cuda.stream(cs):  # capture_begin / _end directly: no device sync, gc or cache flush
            g.capture_begin()  # (its own memory pool, which stays empty: the captured step allocates nothing)
            try:
                body()  # recorded, not executed
            finally:
                g.capture_end()
        torch.cuda.current_stream(st.device).wait_stream(cs)
        st.adam_step = saved
        self._graphs[gkey] = g
        self.live_probe(n)
        return out

    def _build_compact(self, window, global_step, n, n_rays_global, parity, stream):
        """Build slots [ray_offset, ray_offset + n) of ``window`` for ``global_step`` into ray buffer
        ``parity`` on ``stream`` and drop the invalid rays (order kept; one host sync on that stream);
        the global count is all-reduced when data-parallel."""
        b = self._pf_bufs[parity]
        with torch.cuda.stream(stream):
            window.build(L.step_key(self.seed, global_step), self.ray_offset, n, b["rays"][:n], b["dgt"][:n],
                         b["valid"][:n], None, b["far"])
            idx = torch.nonzero(b["valid"][:n]).squeeze(1)
            k = int(idx.numel())  # (the sync)
            slots = idx + self.ray_offset  # (the window slots of the kept rays: the pose gradient's keyframes)
            torch.index_select(b["rays"][:n], 0, idx, out=b["rays_c"][:k])
            torch.index_select(b["dgt"][:n], 0, idx, out=b["dgt_c"][:k])
            cnt = torch.tensor([float(k)], device=self.state.device)
            if self.allreduce is not None:
                self.allreduce(cnt)
            n_glob = int(cnt.item())
            done = torch.cuda.Event()
            done.record(stream)
        return dict(window=window, want=(global_step, n, self.ray_offset, n_rays_global), rays=b["rays_c"][:k],
                    dgt=b["dgt_c"][:k], far=b["far"], n_glob=n_glob, done=done, parity=parity, slots=slots)

