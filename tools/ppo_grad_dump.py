"""Dump the fused minibatch gradient (rx_ppo_minibatch_grad) and one fused update
(rx_ppo_minibatch_update) on ppo_micro.py's seeded inputs, for a bitwise
comparison of two librx builds (same-session A/B of a k_ppo_grad rewrite).

    RX_LIB_PATH=<librx variant> python tools/ppo_grad_dump.py OUT.npz [fp32|bf16] [mb]
    python tools/ppo_grad_dump.py --compare A.npz B.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        ok = all(np.array_equal(a[k], b[k]) for k in a.files)
        diffs = {k: float(np.max(np.abs(a[k] - b[k]))) for k in a.files}
        print({"bit_identical": ok, "max_abs_diff": diffs})
        sys.exit(0 if ok else 1)
    import torch
    from rx.agent import Agent
    from rx.configs import base_config
    from rx.optim import FlatAdam
    from rx.ppo_fused import FusedMinibatchGrad
    from rx.spaces import Box
    out, prec = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fp32"
    mb = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
    D, n_mb = 15, 4
    B = n_mb * mb
    torch.manual_seed(3)
    ag = Agent(Box(-1, 1, (D,)), Box(-1, 1, (2,))).cuda()
    ag.log_std.fill_(-0.8)
    with torch.no_grad():
        ag.actor_mu[4].weight.mul_(30.0)
    fl = FlatAdam(ag, torch.optim.Adam(ag.parameters(), lr=1e-3, eps=1e-5), 0.5)
    g = torch.Generator(device="cuda").manual_seed(0)
    obs = torch.rand(B, D, generator=g, device="cuda") * 2 - 1
    act = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    logp = torch.randn(B, generator=g, device="cuda") * 0.3 - 1.0
    adv = torch.randn(B, generator=g, device="cuda") * 5
    ret = torch.randn(B, generator=g, device="cuda") * 10
    val = ret + torch.randn(B, generator=g, device="cuda") * 0.3
    perm = torch.randperm(B, device="cuda", generator=g)
    fg = FusedMinibatchGrad(ag, fl, (obs, act, logp, adv, ret, val), mb, perm, base_config(kl_target=1e9, policy_dtype=prec))
    fg.adv_stats()
    stop = torch.zeros(1, dtype=torch.bool, device="cuda")
    kl = torch.zeros(1, device="cuda")
    res = {}
    for m in range(n_mb):
        fg.grad(m, stop, kl)
        torch.cuda.synchronize()
        res[f"grad{m}"] = fl.flat_grad.detach().cpu().numpy().copy()
    for m in range(n_mb):  # fused update steps: parameters after each
        fg.update(m, stop, kl)
        torch.cuda.synchronize()
        res[f"param_after{m}"] = fl.flat_param.detach().cpu().numpy().copy()
    np.savez(out, **res)
    print(out, {k: float(np.abs(v).sum()) for k, v in list(res.items())[:2]})


if __name__ == "__main__":
    main()
