"""Multi-rank PPO update logic (rx.dist) with the gloo backend on CPU, world size 2.

Each rank holds half of every minibatch (its env shard).  With one gradient
all-reduce and the 4-float statistics all-reduce per optimizer step, the
ranks must (a) stay bit-identical to each other and (b) match a single
process that sees the union minibatch with the same global normalisation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from rx.configs import base_config
    return base_config(num_envs=8, num_steps=32, num_minibatches=4, update_epochs=2, kl_target=1e9)


def _data(seed=0):
    g = torch.Generator().manual_seed(seed)
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
    from rx.ppo import PPO
    from rx.spaces import Box
    p = PPO.__new__(PPO)
    p.config = cfg
    p.device = torch.device("cpu")
    torch.manual_seed(3)
    p.agent = Agent(Box(-1, 1, shape=(15,)), Box(-1, 1, shape=(2,)))
    # plain SGD here: Adam's m/sqrt(v) turns last-bit gradient differences on
    # near-zero components into +-lr steps, which would test Adam, not the
    # all-reduce (the product keeps Adam, agent/ppo.py:83)
    p.optimizer = torch.optim.SGD(p.agent.parameters(), lr=0.05)
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfg()
        p = _make_ppo(cfg)
        obs, act, logp, adv, ret, val = _data()
        # rank r owns env columns [r*N/2, (r+1)*N/2)
        sl = slice(rank * 4, (rank + 1) * 4)
        np.random.seed(cfg["seed"])
        p.ppo_update(adv[:, sl].contiguous(), ret[:, sl].contiguous(), val[:, sl].contiguous(),
                     logp[:, sl].contiguous(), act[:, sl].contiguous(), obs[:, sl].contiguous())
        q.put((rank, [t.detach().numpy().copy() for t in p.agent.parameters()]))
    finally:
        td.destroy_process_group()


def test_two_rank_update_matches_and_stays_in_sync():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)  # ranks bit-identical after the update
    # single-process reference: same minibatch schedule over the union, global normalisation
    import rx.dist as rd
    cfg = _cfg()
    p = _make_ppo(cfg)
    obs, act, logp, adv, ret, val = _data()
    B = 32 * 8
    mb = cfg["minibatch_size"]
    # rank r's flat index i (over [T, 4]) corresponds to global (t, r*4 + c)
    np.random.seed(cfg["seed"])
    params = list(p.agent.parameters())
    inds = np.arange(B // 2)  # shuffled in place every epoch, as agent/ppo.py:165-168
    for epoch in range(cfg["update_epochs"]):
        np.random.shuffle(inds)
        for s in range(0, B // 2, mb // 2):
            loc = inds[s:s + mb // 2]
            t, c = loc // 4, loc % 4
            gi = np.concatenate([t * 8 + c, t * 8 + 4 + c])
            f = lambda x: x.reshape((B,) + x.shape[2:])[torch.from_numpy(gi)]  # noqa: E731
            _, nl, ent, nv = p.agent.get_action_and_value(f(obs), f(act))
            ratio = (nl - f(logp)).exp()
            a = f(adv)
            a = (a - a.mean()) / (a.std() + 1e-8)
            pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 0.8, 1.2)).mean()
            nv = nv.flatten()
            vc = f(val) + torch.clamp(nv - f(val), -0.2, 0.2)
            vl = 0.5 * torch.max((nv - f(ret)) ** 2, (vc - f(ret)) ** 2).mean()
            loss = pg - cfg["ent_coef"] * ent.mean() + cfg["vf_coef"] * vl
            p.optimizer.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, cfg["max_grad_norm"])
            p.optimizer.step()
    assert rd.world() == 1
    for a, b in zip(res[0], [t.detach().numpy() for t in params]):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


def test_shard_bounds():
    from rx import dist
    assert dist.shard(16) == (0, 16)
    with pytest.raises(ValueError):
        import types
        old = dist.world
        dist.world = lambda: 3  # noqa: E731
        try:
            dist.shard(16)
        finally:
            dist.world = old
        del types


def _seed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rx.dist as rd
        q.put((rank, rd.sampling_seed(1), rd.shard(8)))
    finally:
        td.destroy_process_group()


def test_two_rank_sampling_seeds_differ():
    """Each rank's sampling streams get seed + rank (rank 0 == single process):
    identical noise on every rank would make rank r replay rank 0's envs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict((r, (s, sh)) for r, s, sh in (q.get(timeout=120) for _ in procs))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert res[0][0] == 1 and res[1][0] == 2
    assert res[0][1] == (0, 4) and res[1][1] == (4, 4)


def _capture_worker(rank, world, port, q, fail_rank, bad_replay_rank):
    """rdist.capture_all_or_none with a capture that fails (or a replay that
    disagrees with eager) on ONE rank: every rank must end on the eager form, and
    the eager epochs -- which all-reduce -- must leave the ranks bit-identical."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rx.dist as rd
        w = torch.full((8,), float(rank + 1), dtype=torch.float64)

        def eager_epoch():  # stands in for the shard epoch: local work + a bucket all-reduce
            g = torch.sin(w * 1.7) / world
            td.all_reduce(g)
            w.sub_(0.1 * g)

        def capture():
            if rank == fail_rank:
                raise RuntimeError("capture refused on this rank (test)")
            return "graph"

        def validate(graph):
            return rank != bad_replay_rank

        graph, rec = rd.capture_all_or_none(capture, validate)
        run = eager_epoch if graph is None else (lambda: None)
        w.fill_(1.0)  # the shared state every rank starts the update from
        for _ in range(3):
            run()
        q.put((rank, rec, w.numpy().copy()))
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("fail_rank,bad_replay_rank", [(1, -1), (-1, 0), (-1, -1)])
def test_two_rank_graph_capture_is_all_or_none(fail_rank, bad_replay_rank):
    """the data-parallel epoch graph is used on every rank or on none.
    A capture refused on rank 1, or a replay that disagrees with eager on rank 0,
    puts BOTH ranks on the eager launches (and the ranks stay bit-identical); with
    every rank capturing and validating, both take the graph."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_capture_worker, args=(r, 2, port, q, fail_rank, bad_replay_rank))
             for r in range(2)]
    for pr in procs:
        pr.start()
    res = {r: (rec, w) for r, rec, w in (q.get(timeout=120) for _ in procs)}
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    forms = {res[r][0]["form"] for r in (0, 1)}
    assert len(forms) == 1, res
    want = "graph" if fail_rank < 0 and bad_replay_rank < 0 else "eager"
    assert forms == {want}, res
    if fail_rank >= 0:
        assert res[fail_rank][0]["captured"] is False and res[1 - fail_rank][0]["captured"] is True
        assert all(res[r][0]["all_captured"] is False for r in (0, 1))
    assert np.array_equal(res[0][1], res[1][1])
    if want == "eager":
        assert not np.array_equal(res[0][1], np.ones(8))  # the eager epochs ran
