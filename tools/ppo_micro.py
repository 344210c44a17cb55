"""Same-session A/B timing of the fused PPO minibatch step at configs[1]'s size.

    RX_LIB_PATH=<librx variant> python tools/ppo_micro.py [mb] [fp32|bf16] [label]

Times, with HIP events on the launch stream over 160 back-to-back calls (one
update's 10 epochs x 16 minibatches): rx_ppo_minibatch_grad (k_ppo_grad +
k_ppo_reduce) and rx_ppo_minibatch_update (+ k_adam_apply), KL early stop off,
on a 16-minibatch batch of random rows with a policy that gives non-trivial
ratios.  One JSON line.  Reference: agent/ppo.py:170-207.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))

import torch  # noqa: E402

from rx import _lib  # noqa: E402
from rx.agent import Agent  # noqa: E402
from rx.configs import base_config  # noqa: E402
from rx.optim import FlatAdam  # noqa: E402
from rx.ppo_fused import FusedMinibatchGrad  # noqa: E402
from rx.spaces import Box  # noqa: E402


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    label = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(os.environ.get("RX_LIB_PATH", "librx.so"))
    D, n_mb = 15, 16
    B = n_mb * mb
    torch.manual_seed(3)
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.8)
    with torch.no_grad():
        ag.actor_mu[4].weight.mul_(30.0)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-5, eps=1e-5), 0.5)
    g = torch.Generator(device="cuda").manual_seed(0)
    obs = torch.rand(B, D, generator=g, device="cuda") * 2 - 1
    act = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    logp = torch.randn(B, generator=g, device="cuda") * 0.3 - 1.0
    adv = torch.randn(B, generator=g, device="cuda") * 5
    ret = torch.randn(B, generator=g, device="cuda") * 10
    val = ret + torch.randn(B, generator=g, device="cuda") * 0.3
    perm = torch.randperm(B, device="cuda")
    cfg = base_config(kl_target=1e9, policy_dtype=prec)
    fg = FusedMinibatchGrad(ag, fl, (obs, act, logp, adv, ret, val), mb, perm, cfg)
    fg.adv_stats()
    stop = torch.zeros(1, dtype=torch.bool, device="cuda")
    kl = torch.zeros(1, device="cuda")
    s = torch.cuda.current_stream()
    out = {"label": label, "mb": mb, "precision": prec}
    for name, fn in (("grad", lambda m: fg.grad(m, stop, kl)), ("update", lambda m: fg.update(m, stop, kl))):
        for m in range(n_mb):
            fn(m)
        torch.cuda.synchronize()
        ms = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(160):
                fn(i % n_mb)
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1) / 160 * 1e3)
        out[name + "_us"] = round(min(ms), 2)
        out[name + "_us_all"] = [round(x, 2) for x in ms]
    assert not bool(stop)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
