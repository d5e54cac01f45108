"""GPU: the data-parallel fused PPO update (KL all-reduce before the device-side adaptive LR,
flat-gradient all-reduce scaled inside lgx_adam_clip, global advantage statistics) with two
ranks sharing cuda:0 over gloo, against one process holding both ranks' envs.

Full-batch minibatches (num_mini_batches = 1) so both runs see the same sample sets; same
tolerance rule as test_gpu_ppo.py (Adam normalises gradients at rounding level).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, B, OBS, ACT = 4, 512, 235, 12


def _data(obs=OBS):
    g = torch.Generator().manual_seed(3)
    return dict(obs=torch.randn(T, 2 * B, obs, generator=g), act=torch.randn(T, 2 * B, ACT, generator=g),
                rew=torch.randn(T, 2 * B, 1, generator=g), done=(torch.rand(T, 2 * B, 1, generator=g) < 0.1).byte(),
                val=torch.randn(T, 2 * B, 1, generator=g), logp=torch.randn(T, 2 * B, 1, generator=g) * 0.3 - 17,
                mu=torch.randn(T, 2 * B, ACT, generator=g) * 0.1, sigma=torch.rand(T, 2 * B, ACT, generator=g) * .5 + .75,
                last=torch.randn(2 * B, 1, generator=g))


def _make(n_envs, sl, obs=OBS):
    from legged_gym_amd.rl.actor_critic import ActorCritic
    from legged_gym_amd.rl.ppo import PPO
    torch.manual_seed(0)
    ac = ActorCritic(obs, obs, ACT, [512, 256, 128], [512, 256, 128])
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=1, learning_rate=1e-3, gamma=0.99, lam=0.95,
              schedule="adaptive", entropy_coef=0.01, device="cuda:0")
    assert ppo._fused is not None
    ppo.init_storage(n_envs, T, [obs], [None], [ACT])
    d = _data(obs)
    st = ppo.storage
    for name, key in (("observations", "obs"), ("actions", "act"), ("rewards", "rew"), ("dones", "done"),
                      ("values", "val"), ("actions_log_prob", "logp"), ("mu", "mu"), ("sigma", "sigma")):
        getattr(st, name).copy_(d[key][:, sl])
    st.step = T
    st.compute_returns(d["last"][sl].cuda(), 0.99, 0.95, reduce_stats=ppo._gather_moments)
    return ppo


def _worker(rank, world, port, q, early, obs=OBS):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      LGX_PPO_EARLY_REDUCE=early)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ppo_trace import StepTrace
        ppo = _make(B, slice(rank * B, (rank + 1) * B), obs)
        tr = StepTrace(ppo._fused)
        vl, sl = ppo.update()
        tr.close()
        # early reduction on: two gradient buckets, the first all-reduced from the side stream
        # while dW1 runs; off: one collective after the whole backward
        assert ppo._fused.bucketed == (early == "1")
        assert ppo._fused.join_events == "system"   # peers write the collectives' buffers
        if rank == 0:
            # numpy (pickled by value): CPU tensors would go through shared-memory file descriptors
            # that die with this process
            steps = [{k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in r.items()} for r in tr.steps]
            q.put(([p.detach().cpu().numpy() for p in ppo.actor_critic.parameters()] + [ppo.learning_rate], steps))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("early,obs", [("1", OBS), ("0", OBS), ("1", 48)])
def test_fused_update_two_ranks_equal_one_process(gpu, early, obs):
    """Rank 0's trace of both optimizer steps (tests/ppo_trace.py): the averaged all-reduced
    gradient of step 1 (same parameters in both runs) == the one-process gradient per coordinate
    to 1e-6 + 1e-4 |g| (only the order of the two ranks' partial sums differs), every step ==
    float64 clip + Adam of its gradient (1e-6 + 1e-3 lr), the learning rate sequence identical, and
    at the end all but <= 0.1 % of the coordinates within 1e-5 of the one-process run.
    obs = 48 (Go1 flat): the layer-1 weight gradient is not on lgx_gemm_tn (its padded rows are
    narrower than the 128-column tiles), so db_1 comes from the dA_1 epilogue on the main stream
    and is reduced and all-reduced there (it sat in the side stream's early reduction)."""
    from ppo_trace import StepTrace, adam64
    ref = _make(2 * B, slice(0, 2 * B), obs)
    tr = StepTrace(ref._fused)
    ref.update()
    tr.close()
    if obs != OBS:
        assert 0 not in ref._fused.gemm_dw and 0 not in ref._fused.colsum
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, early, obs)) for r in range(2)]
    for p in procs:
        p.start()
    got, steps = q.get(timeout=300)
    steps = [{k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in r.items()} for r in steps]
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert got[-1] == ref.learning_rate
    assert len(steps) == len(tr.steps) == 2
    assert torch.equal(steps[0]["p0"], tr.steps[0]["p0"].cpu())
    g0, g1 = steps[0]["g"].double(), tr.steps[0]["g"].double().cpu()
    assert ((g0 - g1).abs() <= 1e-6 + 1e-4 * g1.abs()).all(), (g0 - g1).abs().max().item()
    for t, rec in enumerate(steps):
        assert rec["lr"] == tr.steps[t]["lr"]
        p_want, _, _ = adam64(rec, ref.max_grad_norm)
        assert ((rec["p1"].double() - p_want).abs() <= 1e-6 + 1e-3 * rec["lr"]).all(), t
    big = total = 0
    for a, b in zip(got[:-1], ref.actor_critic.parameters()):
        d = np.abs(a - b.detach().cpu().numpy())
        big += int((d > 1e-5).sum())
        total += d.size
    assert big <= 1e-3 * total, (big, total)


@pytest.mark.timeout(280)
def test_bench_two_ranks_self_check(gpu, tmp_path):
    """bench.py --gpus 2 under torch.distributed.run, two ranks sharing cuda:0 over gloo
    (LGX_DIST_BACKEND=gloo; RCCL refuses two ranks on one device): the JSON line carries the
    data-parallel self-check the driver's 8-GPU run is judged by - both ranks seen, bitwise
    identical parameters after the timed iterations (fingerprint spread 0), the two-bucket gradient
    all-reduce taken, event-timed all-reduces."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LGX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", LGX_BENCH_GEMM_TIMING="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--task", "go1_flat_bench", "--num_envs", "256",
           "--no_cpu_baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 512
    dp = d["data_parallel"]
    assert dp["world"] == 2 and dp["backend"] == "gloo" and dp["ranks_seen"] == 2
    assert dp["params_identical_across_ranks"] and dp["param_fingerprint_spread"] == 0
    assert dp["bucketed_allreduce"] is True
    assert dp["allreduce"]["collectives_timed"] >= 2 and dp["allreduce"]["ms_per_iteration"] > 0
    assert dp["join_events"] == "system"   # data-parallel joins keep system-scope events


@pytest.mark.timeout(280)
def test_bench_plain_gpus2_launches_ranks(gpu, tmp_path):
    """`python bench.py --gpus 2` with no launcher: bench.py starts the two ranks
    itself (torch.distributed.run as a child process; gloo so both can share the one test GPU), and
    rank 0's line reports n_gpus 2, both ranks seen and bitwise identical parameters."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(LGX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", LGX_BENCH_GEMM_TIMING="1")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--task", "go1_flat_bench", "--num_envs", "256", "--no_cpu_baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]     # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    dp = d["data_parallel"]
    assert dp["world"] == 2 and dp["ranks_seen"] == 2 and dp["param_fingerprint_spread"] == 0
    assert dp["bucketed_allreduce"] is True


@pytest.mark.timeout(280)
def test_bench_rccl_rehearsal_one_rank(gpu, tmp_path):
    """The RCCL data-parallel path on the test box's one GPU: bench.py under torch.distributed.run
    with ONE rank, backend nccl (= RCCL), LGX_DIST_REHEARSAL=1 so the PPO takes its multi-GPU code
    (parameter broadcast, the two-bucket gradient all-reduce from the side stream while dW1 runs,
    the advantage-statistics and KL all-reduces) over a one-rank communicator - the launch, stream
    and event plumbing the driver's 8-GPU run depends on, which two ranks on one device cannot
    exercise (RCCL refuses duplicate devices)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LGX_DIST_BACKEND="nccl", LGX_DIST_REHEARSAL="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               LGX_BENCH_GEMM_TIMING="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--task", "go1_flat_bench", "--num_envs", "1024",
           "--no_cpu_baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    dp = d["data_parallel"]
    assert dp["world"] == 1 and dp["backend"] == "nccl" and dp["ranks_seen"] == 1
    assert dp["params_identical_across_ranks"] and dp["param_fingerprint_spread"] == 0
    assert dp["join_events"] == "system"
    assert dp["bucketed_allreduce"] is True
    assert dp["allreduce"]["collectives_timed"] >= 2 and dp["allreduce"]["ms_per_iteration"] > 0


def _comm_worker(q):
    """One-rank lgx_comm in a fresh process (RCCL state dies with it)."""
    import ctypes as C
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    torch.cuda.set_device(0)
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    path = path.encode() if os.path.exists(path) else None
    uid = (C.c_uint8 * 128)()
    lgxlib.check(lib.lgx_comm_unique_id(path, uid), "comm_unique_id")
    comm = C.c_void_p()
    lgxlib.check(lib.lgx_comm_create(path, uid, 1, 0, 0, C.byref(comm)), "comm_create")
    x = torch.randn(1 << 20, device="cuda:0")
    want = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    for op in (0, 1):   # sum, average over one rank: the identity
        lgxlib.check(lib.lgx_allreduce_grads(comm, C.c_void_p(x.data_ptr()), x.numel(), op,
                                             C.c_void_p(s.cuda_stream)), "allreduce_grads")
    s.synchronize()
    ok = bool(torch.equal(x, want))
    bad = lib.lgx_allreduce_grads(comm, C.c_void_p(x.data_ptr()), x.numel(), 7, C.c_void_p(s.cuda_stream))
    lgxlib.check(lib.lgx_comm_destroy(comm), "comm_destroy")
    q.put((ok, bad))


@pytest.mark.timeout(200)
def test_lgx_comm_one_rank_allreduce(gpu):
    """lgx_comm_create / lgx_allreduce_grads over a one-rank RCCL communicator on the caller's
    stream (RCCL refuses two ranks on one device): sum and average leave the buffer bitwise
    unchanged; an unknown op is refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_comm_worker, args=(q,))
    p.start()
    ok, bad = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0 and ok and bad == -1


def _native_worker(port, q):
    """One-rank nccl group (LGX_DIST_REHEARSAL=1): the same update with torch.distributed's
    all-reduce and with lgx_allreduce_grads, from the same state, in one process."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      LGX_DIST_REHEARSAL="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        out = {}
        for native in ("0", "1"):
            os.environ["LGX_NATIVE_ALLREDUCE"] = native
            ppo = _make(2 * B, slice(0, 2 * B))
            assert ppo._fused is not None and ppo.dist is not None
            ppo.update()
            out[native] = ([p.detach().cpu().numpy() for p in ppo.actor_critic.parameters()],
                           ppo.learning_rate, ppo._fused.allreduce_impl, ppo._fused.bucketed)
            ppo._fused.close_comm()
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(200)
def test_native_allreduce_update_matches_torch_allreduce(gpu):
    """The data-parallel update over a one-rank RCCL group: with LGX_NATIVE_ALLREDUCE=1 the
    gradient buckets go through lgx_allreduce_grads on the update's own streams (the main-stream
    bucket ordered after the side-stream one by an event), and the parameters
    and learning rate after the update are bitwise those of the torch.distributed path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    (pt, lrt, it, _), (pn, lrn, inn, bn) = out["0"], out["1"]
    assert it == "torch" and inn == "lgx"
    assert bn   # (two buckets: collectives from the side and the main stream on one communicator)
    assert lrt == lrn
    for a, b in zip(pt, pn):
        assert np.array_equal(a, b)


@pytest.mark.timeout(280)
def test_bench_rccl_rehearsal_native_allreduce(gpu, tmp_path):
    """bench.py's one-rank RCCL rehearsal with LGX_NATIVE_ALLREDUCE=1 reports the native all-reduce
    (event-timed, both buckets) and the data-parallel self-check."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LGX_DIST_BACKEND="nccl", LGX_DIST_REHEARSAL="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               LGX_BENCH_GEMM_TIMING="1", LGX_NATIVE_ALLREDUCE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--task", "go1_flat_bench", "--num_envs", "1024",
           "--no_cpu_baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    dp = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["data_parallel"]
    assert dp["allreduce_impl"] == "lgx" and dp["ranks_seen"] == 1 and dp["param_fingerprint_spread"] == 0
    assert dp["bucketed_allreduce"] is True and dp["allreduce"]["collectives_timed"] >= 2


def _rec_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ppo = _make_rec(B, slice(rank * B, (rank + 1) * B))
        assert ppo._fused is not None and ppo._fused.recurrent and ppo.dist is not None
        ppo.update()
        if rank == 0:
            q.put([p.detach().cpu().numpy() for p in ppo.actor_critic.parameters()] + [ppo.learning_rate])
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _make_rec(n_envs, sl):
    """ActorCriticRecurrent + PPO with the storage of envs `sl` of one fixed rollout (observations,
    dones, saved LSTM states, returns) - the same data in the one-process and the per-rank runs."""
    from legged_gym_amd.rl.actor_critic import ActorCriticRecurrent
    from legged_gym_amd.rl.ppo import PPO
    torch.manual_seed(0)
    ac = ActorCriticRecurrent(48, 48, ACT, [512, 256, 128], [512, 256, 128], rnn_hidden_size=64)
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=1, learning_rate=1e-3, gamma=0.99, lam=0.95,
              schedule="adaptive", entropy_coef=0.01, device="cuda:0")
    ppo.init_storage(n_envs, T, [48], [None], [ACT])
    g = torch.Generator().manual_seed(5)
    d = dict(obs=torch.randn(T, 2 * B, 48, generator=g), act=torch.randn(T, 2 * B, ACT, generator=g),
             rew=torch.randn(T, 2 * B, 1, generator=g), done=(torch.rand(T, 2 * B, 1, generator=g) < 0.2).byte(),
             val=torch.randn(T, 2 * B, 1, generator=g), logp=torch.randn(T, 2 * B, 1, generator=g) * 0.3 - 17,
             mu=torch.randn(T, 2 * B, ACT, generator=g) * 0.1, sigma=torch.rand(T, 2 * B, ACT, generator=g) * .5 + .75,
             h=torch.randn(T, 1, 2 * B, 64, generator=g) * 0.5, c=torch.randn(T, 1, 2 * B, 64, generator=g),
             last=torch.randn(2 * B, 1, generator=g))
    st = ppo.storage
    for name, key in (("observations", "obs"), ("actions", "act"), ("rewards", "rew"), ("dones", "done"),
                      ("values", "val"), ("actions_log_prob", "logp"), ("mu", "mu"), ("sigma", "sigma")):
        getattr(st, name).copy_(d[key][:, sl])
    # the memories' states before every step (LSTM: h, c), actor and critic
    st.saved_hidden_states_a = [d["h"][:, :, sl].cuda().contiguous(), d["c"][:, :, sl].cuda().contiguous()]
    st.saved_hidden_states_c = [x.clone() for x in st.saved_hidden_states_a]
    st.step = T
    st.compute_returns(d["last"][sl].cuda(), 0.99, 0.95, reduce_stats=ppo._gather_moments)
    return ppo


def test_fused_recurrent_update_two_ranks_equal_one_process(gpu):
    """The fused recurrent update data-parallel (two gloo ranks on cuda:0, one gradient all-reduce
    after the memories' autograd backward) against one process holding both ranks' envs: same
    learning rate, all but <= 0.1 % of the coordinates within 1e-5 after two epochs."""
    ref = _make_rec(2 * B, slice(0, 2 * B))
    assert ref._fused is not None and ref._fused.recurrent
    ref.update()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rec_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert got[-1] == ref.learning_rate
    big = total = 0
    for a, b in zip(got[:-1], ref.actor_critic.parameters()):
        d = np.abs(a - b.detach().cpu().numpy())
        big += int((d > 1e-5).sum())
        total += d.size
    assert big <= 1e-3 * total, (big, total)
