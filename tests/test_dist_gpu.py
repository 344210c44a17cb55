"""Data-parallel PPO update on the device path (FlatAdam + rx_adam_clip_step,
one flat-gradient all-reduce per optimizer step), 2 ranks sharing one GPU
over gloo (the GPU box has one device; RCCL needs one GPU per rank).  Ranks
must stay bit-identical and match one process over the union minibatch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(fused=False):
    from rx.configs import base_config
    return base_config(num_envs=8, num_steps=32, num_minibatches=4, update_epochs=2, kl_target=1e9,
                       fused_update=fused)


def _data():
    g = torch.Generator().manual_seed(0)
    T, N = 32, 8
    obs = torch.rand(T, N, 15, generator=g) * 2 - 1
    act = torch.rand(T, N, 2, generator=g) * 2 - 1
    logp = torch.randn(T, N, generator=g) - 2
    adv = torch.randn(T, N, generator=g) * 5
    ret = torch.randn(T, N, generator=g) * 10
    val = torch.randn(T, N, generator=g) * 10
    return obs, act, logp, adv, ret, val


def _make_ppo(cfg):
    from rx.agent import Agent
    from rx.optim import FlatAdam
    from rx.ppo import PPO
    from rx.spaces import Box
    p = PPO.__new__(PPO)
    p.config = cfg
    p.device = torch.device("cuda")
    torch.manual_seed(3)
    p.agent = Agent(Box(-1, 1, shape=(15,)), Box(-1, 1, shape=(2,))).cuda()
    p.optimizer = torch.optim.Adam(p.agent.parameters(), lr=3e-4, eps=1e-5)
    p._flat = FlatAdam(p.agent, p.optimizer, cfg["max_grad_norm"])
    return p


def _worker(rank, world, port, q, fused):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfg(fused)
        p = _make_ppo(cfg)
        sl = slice(rank * 4, (rank + 1) * 4)
        d = [t[:, sl].contiguous().cuda() for t in _data()]
        obs, act, logp, adv, ret, val = d
        np.random.seed(cfg["seed"])
        p.ppo_update(adv, ret, val, logp, act, obs)
        q.put((rank, p._flat.flat_param.cpu().numpy().copy(), float(p._flat.step_t)))
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("fused", [False, True], ids=["autograd", "fused_shard"])
def test_two_rank_flat_update_in_sync(fused):
    """fused: the HIP shard path (rx_ppo_minibatch_grad_shard + ONE bucket
    all-reduce per step); autograd: torch autograd + flat-gradient all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, fused)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict((r, (a, s)) for r, a, s in (q.get(timeout=300) for _ in procs))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert np.array_equal(res[0][0], res[1][0])  # ranks bit-identical
    cfg = _cfg()
    assert res[0][1] == cfg["update_epochs"] * cfg["num_minibatches"]
    # single process, same minibatch schedule over the union, global normalisation
    import rx.dist as rd
    p = _make_ppo(cfg)
    obs, act, logp, adv, ret, val = [t.cuda() for t in _data()]
    B, mb = 32 * 8, cfg["minibatch_size"]
    np.random.seed(cfg["seed"])
    inds = np.arange(B // 2)
    b = p._flat_batch(adv, ret, val, logp, act, obs)
    p._flat.sync_lr()
    for epoch in range(cfg["update_epochs"]):
        np.random.shuffle(inds)
        for s in range(0, B // 2, mb // 2):
            loc = inds[s:s + mb // 2]
            t, c = loc // 4, loc % 4
            gi = torch.from_numpy(np.concatenate([t * 8 + c, t * 8 + 4 + c])).cuda()
            loss, _ = p._minibatch_loss(b, gi)
            p._flat.zero_grad()
            loss.backward()
            p._flat.step()
    assert rd.world() == 1
    np.testing.assert_allclose(res[0][0], p._flat.flat_param.cpu().numpy(), rtol=1e-4, atol=1e-5)


def _noise_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = _make_ppo(_cfg(True))  # torch.manual_seed(3) -> identical initial policy on every rank
        p._seed_sampling()
        eps = torch.empty(64, 2, device="cuda").normal_()
        q.put((rank, eps.cpu().numpy(), p._flat.flat_param.cpu().numpy()))
    finally:
        td.destroy_process_group()


def test_two_rank_action_noise_differs():
    """PPO._seed_sampling: same initial parameters on every rank, different
    action-noise streams (rank 0's == the single-process stream of config seed)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_noise_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict((r, (e, w)) for r, e, w in (q.get(timeout=300) for _ in procs))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1])
    assert not np.array_equal(res[0][0], res[1][0])
    torch.manual_seed(_cfg()["seed"])
    want = torch.empty(64, 2, device="cuda").normal_()
    assert np.array_equal(res[0][0], want.cpu().numpy())


def _rccl_worker(port, q):
    """One rank, process group over RCCL ("nccl") on cuda:0: the fused shard update
    with every bucket / moment all-reduce a real RCCL all_reduce on device memory
    (rx.dist.all_reduce_sum is replaced, since rx.dist.active() is False at world 1)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    import rx.dist as rd
    from tests.test_optim_gpu import _rollout
    from tests.test_ppo_fused_gpu import _trainer
    torch.cuda.set_device(0)
    td.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert td.get_backend() == "nccl"
        calls = {"n": 0, "bytes": 0, "dev": True}

        def rccl_sum(t):
            calls["n"] += 1
            calls["bytes"] += t.numel() * t.element_size()
            calls["dev"] &= t.is_cuda
            td.all_reduce(t)  # RCCL, on its own stream, ordered after librx's launches on the current one
            return t

        res = []
        eager_calls = None
        for shard, graph in ((False, False), (True, False), (True, True)):
            t = _trainer(graph_update=False, shard_update=shard, graph_dp=graph, kl_target=1e9)
            data = _rollout(t)
            np.random.seed(4)
            saved = rd.all_reduce_sum
            if shard:
                rd.all_reduce_sum = rccl_sum
            try:
                for u in range(2):
                    t._anneal(u, 4)
                    t.ppo_update(*data)
            finally:
                rd.all_reduce_sum = saved
            torch.cuda.synchronize()
            res.append((t._flat.flat_param.cpu().numpy().copy(), t._flat.exp_avg.cpu().numpy().copy(),
                        float(t._flat.step_t)))
            if shard and not graph:
                eager_calls = dict(calls)
            c = t.config
        graph_dp = dict(rd.GRAPH_DP)
        ver = ".".join(str(v) for v in torch.cuda.nccl.version())
        q.put((res, eager_calls, c["update_epochs"], c["num_minibatches"], ver, graph_dp))
    finally:
        td.destroy_process_group()


def test_rccl_world1_shard_update_equals_fused():
    """RCCL executed: init_process_group("nccl") at world size 1,
    the data-parallel launch sequence (adv moments -> RCCL all-reduce -> finalize;
    per optimizer step rx_ppo_minibatch_grad_shard -> RCCL all-reduce of
    FlatAdam.bucket -> rx_ppo_kl_check -> rx_adam_clip_step) over two updates ==
    the single-rank fused update bit for bit.  The stream ordering between the
    librx launches on torch's current stream and RCCL's collective is what the
    8-GPU run relies on."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    pr.start()
    res, calls, E, n_mb, ver, graph_dp = q.get(timeout=600)
    pr.join(timeout=120)
    assert pr.exitcode == 0
    (pa, ma, sa), (pb, mb_, sb), (pc, mc, sc) = res
    assert calls["dev"] and calls["n"] == 2 * E * (n_mb + 1)  # per update: E moment + E * n_mb bucket all-reduces
    assert sa == sb == sc == 2 * E * n_mb
    assert np.array_equal(pa, pb) and np.array_equal(ma, mb_)
    # the data-parallel epoch captured as ONE HIP graph, RCCL all-reduces
    # included (graph_dp), replayed == eager == the single-rank fused update
    # (rdist.capture_all_or_none: captured on every rank, first replay == eager epoch bit for bit)
    assert graph_dp["captured"] is True and graph_dp["form"] == "graph" and graph_dp["all_validated"], graph_dp
    assert np.array_equal(pa, pc) and np.array_equal(ma, mc)
    print(f"\nRCCL {ver}: {calls['n']} all-reduces, {calls['bytes']} B, shard update (eager and one graph per "
          "epoch) == fused bit for bit")
