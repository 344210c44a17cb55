"""Data parallelism over GPUs (BASELINE.json configs[4]).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Envs
are independent, so each rank owns the contiguous env shard
[rank*N/W, (rank+1)*N/W) with its own track table, rollout buffer and GAE;
the only exchanges are, per optimizer step,

* one all-reduce of the flat gradient bucket (10,563 floats = 42 KB for the
  15-dim policy) -- latency-bound on xGMI, so ONE bucket, never per-parameter;
* one 4-float all-reduce [KL sum, advantage sum, advantage square-sum, count]
  so the KL early stop and the minibatch advantage normalisation are global
  (every rank stops in the same minibatch);

with the fused HIP update (rx.ppo_fused.FusedMinibatchGrad.shard_epoch) the
same exchanges shrink to ONE all-reduce per optimizer step of the bucket
[flat gradient / W, KL / W] (FlatAdam.bucket) plus one per epoch of every
minibatch's advantage (sum, square-sum);

and one 3-float all-reduce of episode statistics per update.  Minibatch
shuffles use np.random with the same seed on every rank, so all ranks walk
the same minibatch schedule over their own shards.

Everything here also runs with the gloo backend on CPU (tests/test_dist_cpu.py).
"""
import torch
import torch.distributed as td


# all-reduces issued through this module (count, payload bytes): bench.py reports
# the per-update figures of its data-parallel PPO leg from these
COUNTS = {"all_reduce": 0, "bytes": 0}


def _all_reduce(t, **kw):
    COUNTS["all_reduce"] += 1
    COUNTS["bytes"] += t.numel() * t.element_size()
    td.all_reduce(t, **kw)


def active():
    return td.is_available() and td.is_initialized() and td.get_world_size() > 1


def world():
    return td.get_world_size() if active() else 1


def rank():
    return td.get_rank() if active() else 0


def shard(n):
    """(first env, env count) of this rank's shard of n envs."""
    w, r = world(), rank()
    if n % w:
        raise ValueError(f"num_envs={n} is not divisible by world size {w}")
    k = n // w
    return r * k, k


def sampling_seed(seed):
    """Seed of this rank's sampling streams (action noise, device shuffles,
    random opponents): seed + rank, so rank 0 equals the single-process run
    and no two ranks draw the same noise.  The initial policy stays shared
    (every rank seeds its init with ``seed``)."""
    return int(seed) + rank()


def sum_stats(s, device):
    """Sum (sum_return, sum_length, count) over ranks."""
    if not active():
        return s
    t = torch.tensor([float(s[0]), float(s[1]), float(s[2])], dtype=torch.float64, device=device)
    _all_reduce(t)
    return float(t[0]), float(t[1]), int(round(float(t[2])))


def minibatch_stats(kl_sum, adv):
    """[KL sum, sum(adv), sum(adv^2), count] over all ranks' minibatch shards."""
    a = adv.detach().to(torch.float64)
    t = torch.stack([kl_sum.detach().to(torch.float64), a.sum(), (a * a).sum(),
                     torch.tensor(float(adv.numel()), dtype=torch.float64, device=adv.device)])
    if active():
        _all_reduce(t)
    return t


def average_gradients(params):
    """Mean of every gradient over ranks: ONE flat bucket, one all-reduce."""
    if not active():
        return
    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    _all_reduce(flat)
    flat.div_(td.get_world_size())
    o = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[o:o + n].view_as(g))
        o += n


def average_flat(flat):
    """Mean over ranks of the flat gradient buffer (rx.optim.FlatAdam): one all-reduce, no copies."""
    if not active():
        return
    _all_reduce(flat)
    flat.div_(td.get_world_size())


# bench.py's world-size-1 RCCL leg: issue the collectives through a 1-rank process
# group anyway, so the data-parallel update's launch / collective sequence is priced
# on one GPU
FORCE_COLLECTIVES = {"on": False}
# the last data-parallel epoch graph decision (rx.ppo, capture_all_or_none): this rank's
# capture, the cross-rank agreement, the replay-vs-eager validation, the refusal
GRAPH_DP = {"captured": None, "error": None}


def agree(ok, device=None):
    """True iff ``ok`` holds on EVERY rank (one MIN all-reduce of a flag; on the
    device for RCCL, on the host for gloo).  Not counted in COUNTS: it runs once
    per captured epoch form, outside the update's steady state."""
    if not active():
        return bool(ok)
    dev = device if (td.get_backend() == "nccl" and device is not None) else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    td.all_reduce(t, op=td.ReduceOp.MIN)
    return bool(int(t.item()))


def capture_all_or_none(capture, validate=None, device=None):
    """The data-parallel epoch's launch form, decided for ALL ranks at once.

    ``capture()`` records the epoch (collectives included) as a HIP graph and
    returns it, or raises; ``validate(graph)`` (optional) replays it against the
    eager epoch on the same state and returns whether they agree bit for bit.
    Every rank then learns, by one MIN all-reduce per stage, whether every rank
    captured (and validated): if any did not, EVERY rank runs the eager epoch, so
    no two ranks ever issue the same collectives from different launch forms.
    -> (graph or None, record); the record also lands in GRAPH_DP."""
    graph, err = None, None
    try:
        graph = capture()
        ok = graph is not None
    except Exception as e:  # noqa: BLE001 -- recorded; the ranks agree on eager below
        ok, err = False, f"{type(e).__name__}: {e}"[:300]
    rec = {"captured": ok, "error": err, "rank": rank(), "world": world()}
    ok = agree(ok, device)
    rec["all_captured"] = ok
    if ok and validate is not None:
        try:
            v = bool(validate(graph))
        except Exception as e:  # noqa: BLE001
            v, rec["error"] = False, f"validate: {type(e).__name__}: {e}"[:300]
        rec["validated"] = v
        ok = agree(v, device)
        rec["all_validated"] = ok
    rec["form"] = "graph" if ok else "eager"
    GRAPH_DP.clear()
    GRAPH_DP.update(rec)
    return (graph if ok else None), rec


def capturable():
    """Collectives of this process group can be recorded in a HIP graph: RCCL
    ("nccl") can, gloo (host-side) cannot; no group at all: nothing to record."""
    if not (td.is_available() and td.is_initialized()):
        return True
    return td.get_backend() == "nccl"


def all_reduce_sum(t):
    """In-place SUM over ranks (the fused data-parallel update pre-scales its
    shard gradient and KL by 1/world, so the sum is the global mean)."""
    if active() or (FORCE_COLLECTIVES["on"] and td.is_available() and td.is_initialized()):
        _all_reduce(t)
    return t


def broadcast_parameters(module, src=0):
    """Make every rank start from rank ``src``'s weights."""
    if not active():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        td.broadcast(t.data, src)
