"""The data-parallel StepEngine through a real torch.distributed backend: two processes (gloo, both
on GPU 0) each step their shard with the bucketed, asynchronous gradient all-reduce
(``allreduce(t, async_op=True)``, two level-range buckets by default (LONER_AR_BUCKETS: levels 8-15,
then 0-7 with the MLP), each exchanged while the next accumulates) and must
reproduce the single-engine gradient, with bit-identical parameters on both replicas (SURVEY.md
§8(e)).  The driver's multi-GPU runs use the same code path over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

L2JS = dict(loss_selection="L2_JS", JS_loss=dict(min_js_score=1.0, max_js_score=10.0, alpha=1.0),
            decay_los_lambda=False, los_lambda=1000.0, min_los_lambda=10.0, los_lambda_decay_rate=0.001,
            los_lambda_decay_steps=15000, decay_depth_eps=True, depth_eps=3.0, min_depth_eps=0.5,
            depth_eps_decay_rate=0.95, depth_eps_decay_steps=1, depthloss_lambda=0.005)


def _setup():
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    win = syn.make_window("forest", n_kf=2, seed=3)
    rays, dgt = syn.build_batch(win, "forest", rays_per_kf=40, sky_per_kf=8, strategy="MASK", seed=1)
    cfg = S_.StepConfig(n_samples=512, occ_lr=1e-3, loss=S_.LossConfig.from_dict(L2JS))
    st = S_.FieldState(cfg, device="cuda:0", table_init=0.5, seed=5)
    st.params[2048:3072].mul_(40.0)
    st.refresh_shadow()
    return S_, syn, rays.cuda(), dgt.cuda(), st


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from loner_amd.shard import shard_range
    S_, syn, rays, dgt, st = _setup()
    R = rays.shape[0]
    s0, s1 = shard_range(R, rank, world)

    def allreduce(t, async_op=False):
        return dist.all_reduce(t, async_op=async_op)

    eng = S_.StepEngine(st, s1 - s0, seed=9, allreduce=allreduce, ray_offset=s0)
    for k in range(2):
        eng.step(rays[s0:s1].contiguous(), dgt[s0:s1].contiguous(), global_step=3 + k, scale=syn.CUBES["forest"][0],
                 far_ref=float(rays[0, -1]), n_rays_global=R)
    torch.cuda.synchronize()
    np.save(os.path.join(out, f"grad{rank}.npy"), st.grad.cpu().numpy())
    np.save(os.path.join(out, f"params{rank}.npy"), st.params.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_bucketed_async_allreduce(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    S_, syn, rays, dgt, st = _setup()
    eng = S_.StepEngine(st, rays.shape[0], seed=9)
    for k in range(2):
        eng.step(rays, dgt, global_step=3 + k, scale=syn.CUBES["forest"][0], far_ref=float(rays[0, -1]))
    g_ref = st.grad.cpu().numpy()
    p0, p1 = (np.load(tmp_path / f"params{r}.npy") for r in range(2))
    g0 = np.load(tmp_path / "grad0.npy")
    assert np.array_equal(p0, p1)
    assert np.linalg.norm(g0 - g_ref) / np.linalg.norm(g_ref) < 1e-4
    # every bucket carried its share: the MLP block and each level range match the single engine
    for a, b in [(0, st.n_mlp)] + [(st.n_mlp + 2 * int(st.desc.offset[l0]), st.n_mlp + 2 * int(st.desc.offset[l1]))
                                   for l0, l1 in eng.ar_groups]:
        assert np.linalg.norm(g0[a:b] - g_ref[a:b]) <= 1e-4 * np.linalg.norm(g_ref[a:b]) + 1e-12


def _zero_worker(rank, world, port, out):
    import torch.distributed as dist
    # the level-looped scatter (and with it the live backward) at this small batch too (read at every launch)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LONER_SCATTER_ROWS_MIN="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from loner_amd.shard import shard_range

    def allreduce(t, async_op=False):
        return dist.all_reduce(t, async_op=async_op)

    hooks = dict(reduce_scatter=lambda o, i, async_op=False: dist.reduce_scatter_tensor(o, i, async_op=async_op),
                 all_gather=lambda o, i, async_op=False: dist.all_gather_into_tensor(o, i, async_op=async_op))
    # the exchange on two communicators (bench.py's default, LONER_EXCHANGE_GROUPS=2): the all-gathers on a group
    # of their own, so a range's gather runs beside the next range's reduce-scatter
    ag_group = dist.new_group(list(range(world)))
    hooks2 = dict(reduce_scatter=hooks["reduce_scatter"],
                  all_gather=lambda o, i, async_op=False: dist.all_gather_into_tensor(o, i, group=ag_group,
                                                                                     async_op=async_op))
    for tag, zero, hk, live, ert in (("ar", None, {}, False, False), ("zero", (rank, world), hooks, False, False),
                                     ("zero2", (rank, world), hooks2, False, False), ("arlive", None, {}, True, False),
                                     ("zero2live", (rank, world), hooks2, True, False),
                                     ("zero2ert", (rank, world), hooks2, True, True)):
        S_, syn, rays, dgt, st = _setup()
        R = rays.shape[0]
        s0, s1 = shard_range(R, rank, world)
        eng = S_.StepEngine(st, s1 - s0, seed=9, allreduce=allreduce, ray_offset=s0, zero=zero, **hk)
        eng.live_bwd, eng._live = live, live
        eng.ert = ert  # early ray termination at the fixed cuts through the sharded exchange
        for k in range(3):
            eng.step(rays[s0:s1].contiguous(), dgt[s0:s1].contiguous(), global_step=9 + k, scale=syn.CUBES["forest"][0],
                     far_ref=float(rays[0, -1]), n_rays_global=R)
        eng.sync_master()
        torch.cuda.synchronize()
        np.save(os.path.join(out, f"{tag}_params{rank}.npy"), st.params.cpu().numpy())
        np.save(os.path.join(out, f"{tag}_shadow{rank}.npy"), st.shadow.cpu().numpy())
        np.save(os.path.join(out, f"{tag}_m{rank}.npy"), st.m.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_sharded_optimizer(tmp_path):
    """ZeRO-1 (reduce-scatter of each level range's gradient, Adam on each rank's half, all-gather of the
    fp16 shadow) gives the all-reduce path's parameters bit for bit, on both ranks, over 3 steps (one an
    OGM step); after sync_master the fp32 master and the moments agree too.  The same with the all-gathers
    on a second process group (two communicators: the exchange's reduce-scatters and gathers unserialised)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_zero_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for what in ("params", "shadow", "m"):
        ref = np.load(tmp_path / f"ar_{what}0.npy")
        assert np.array_equal(ref, np.load(tmp_path / f"ar_{what}1.npy"))
        for r in range(2):
            assert np.array_equal(ref, np.load(tmp_path / f"zero_{what}{r}.npy")), (what, r)
            assert np.array_equal(ref, np.load(tmp_path / f"zero2_{what}{r}.npy")), (what, r)
            # the live backward (records only for samples with dL/dsigma != 0; ignored where the level-looped scatter
            # does not apply) through both exchanges: bitwise the same
            assert np.array_equal(ref, np.load(tmp_path / f"arlive_{what}{r}.npy")), (what, r)
            assert np.array_equal(ref, np.load(tmp_path / f"zero2live_{what}{r}.npy")), (what, r)
            # and with early ray termination on top (the phases over the rays still alive): bitwise the same
            assert np.array_equal(ref, np.load(tmp_path / f"zero2ert_{what}{r}.npy")), (what, r)


def _pipe_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow

    def allreduce(t, async_op=False):
        return dist.all_reduce(t, async_op=async_op)

    win = RayWindow(syn.make_window("forest", 2 * world, seed=4), syn.world_cube("forest"),
                    syn.SENSORS["forest"]["ray_range"], n_lidar=128, n_sky=16, strategy="MASK", device="cuda:0")
    assert win.all_valid
    R = win.n_slots // world
    for pipeline in (False, True):
        st = S_.FieldState(S_.StepConfig(n_samples=128, occ_lr=1e-3), device="cuda:0", table_init=0.5, seed=5)
        eng = S_.StepEngine(st, R, seed=9, allreduce=allreduce, ray_offset=rank * R)
        eng.pipeline = pipeline
        zs = []
        for g in (8, 9, 10, 11, 12):  # step 10 updates the OGM; 11's prefetched sampling must see the update
            eng.step_window(win, global_step=g, n_rays_global=win.n_slots)
            zs.append(eng.z.clone())
        eng.finish()
        torch.cuda.synchronize()
        np.save(os.path.join(out, f"pipe{int(pipeline)}_occ{rank}.npy"), st.occ.cpu().numpy())
        np.save(os.path.join(out, f"pipe{int(pipeline)}_z{rank}.npy"), torch.stack(zs).cpu().numpy())
        np.save(os.path.join(out, f"pipe{int(pipeline)}_params{rank}.npy"), st.params.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_pipelined_ogm_equals_plain(tmp_path):
    """The data-parallel OGM update is asynchronous (its SGD step lands before the grid's next reader): with the
    eager path's pipeline (step k + 1's sampling prefetched on a side stream) the occupancy grid, the samples of
    the steps after the OGM step and the parameters are bit for bit those of LONER_PIPELINE=0, on both ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(2):
        for what in ("occ", "z", "params"):
            assert np.array_equal(np.load(tmp_path / f"pipe0_{what}{r}.npy"), np.load(tmp_path / f"pipe1_{what}{r}.npy")), \
                (what, r)


def test_sharded_optimizer_emulation_single_process():
    """One process with zero=(0, N) and no collectives (bench.py --shard-of): Adam touches exactly this
    rank's chunk of every level range, identically to the full Adam there."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    S_, syn, rays, dgt, st = _setup()
    p0 = st.params.clone()
    eng = S_.StepEngine(st, rays.shape[0], seed=9, zero=(0, 4))
    eng.step(rays, dgt, global_step=3, scale=syn.CUBES["forest"][0], far_ref=float(rays[0, -1]))
    S2, _, _, _, st2 = _setup()
    eng2 = S2.StepEngine(st2, rays.shape[0], seed=9)
    eng2.step(rays, dgt, global_step=3, scale=syn.CUBES["forest"][0], far_ref=float(rays[0, -1]))
    torch.cuda.synchronize()
    for a0, a1, c in eng.zero_chunks:
        assert torch.equal(st.params[a0:a0 + c], st2.params[a0:a0 + c])
        assert torch.equal(st.params[a0 + c:a1], p0[a0 + c:a1])  # the other ranks' chunks: untouched here
