"""Batched evaluation -- evaluate.py:12-66,173-238 and utils/metrics.py:39-78.

The reference evaluates a policy on 40 tracks (gen_tracks(40, seed=42)) x 5
runs, run r using width RandomState(42+r).randint(4, 10) (note: indexed by
RUN, evaluate.py:30), one episode at a time with a batch-1 stochastic policy
for at most 2,000 steps.  Here all 200 episodes run at once as one device
vector env with autoreset disabled; each env's metrics freeze at its first
terminal step.  ``success_rate`` = finished / episodes (evaluate.py:54) is
the quantity behind "PPO wall-clock to 90% success" (BASELINE.json metric).

Reference quirk kept: gen_tracks(seed=42) draws the FIRST track's parameters
from whatever state the global numpy RNG is in (evaluate.py never seeds it);
``eval_pool`` takes an explicit ``global_seed`` for that draw (default 0) and
restores the caller's RNG state afterwards.
"""
import numpy as np
import torch

from .track import gen_tracks


def eval_pool(num_tracks=40, num_runs=5, seed=42, global_seed=0):
    state = np.random.get_state()
    try:
        np.random.seed(global_seed)
        pool = gen_tracks(num_tracks=num_tracks, seed=seed)
    finally:
        np.random.set_state(state)
    widths = [np.random.RandomState(seed + i).randint(4, 10) for i in range(num_tracks)]
    cps, ws, ids = [], [], []
    for t in range(num_tracks):
        for r in range(num_runs):
            cps.append(pool[t])
            ws.append(widths[r])  # evaluate.py:30 indexes widths by run
            ids.append((t, r))
    return cps, ws, ids


class Evaluator:
    """Reusable 200-episode evaluation env (evaluate.py protocol)."""

    def __init__(self, num_tracks=40, num_runs=5, seed=42, global_seed=0, max_steps=2000, device=None,
                 n_sensors=11):
        from .vector_env import RacingVectorEnv
        cps, ws, self.ids = eval_pool(num_tracks, num_runs, seed, global_seed)
        self.max_steps = max_steps
        self.venv = RacingVectorEnv(cps, ws, n_agents=1, n_sensors=n_sensors, device=device, autoreset="disabled")
        self.device = self.venv.device

    @torch.no_grad()
    def run(self, agent, deterministic=False):
        """utils/metrics.py:39-78 for every episode at once; returns evaluate.py's summary dict."""
        v = self.venv
        N = v.num_envs
        dev = self.device
        obs = v.reset_device()
        active = torch.ones(N, dtype=torch.bool, device=dev)
        total_reward = torch.zeros(N, dtype=torch.float64, device=dev)
        total_dist = torch.zeros(N, dtype=torch.float64, device=dev)
        steps = torch.zeros(N, dtype=torch.int64, device=dev)
        fin = torch.zeros(N, dtype=torch.bool, device=dev)
        crash = torch.zeros(N, dtype=torch.bool, device=dev)
        prog = torch.zeros(N, dtype=torch.float64, device=dev)
        speed = torch.zeros(N, dtype=torch.float64, device=dev)
        x, y = v.state["x"], v.state["y"]
        px, py = x.clone(), y.clone()
        first = True
        for t in range(self.max_steps):
            if deterministic:
                a = agent.actor_mu(obs).clamp(-1.0, 1.0)
            else:
                a = agent.get_action_and_value(obs)[0]
            obs, _, done = v.step_device(a, full_info=True)
            r64 = v.buf["reward64"]
            info = v.buf["info"][:, 0]
            total_reward += torch.where(active, r64, torch.zeros_like(r64))
            if not first:  # metrics.py:59-64: distance between consecutive post-step positions
                d = torch.sqrt((x - px) ** 2 + (y - py) ** 2)
                total_dist += torch.where(active, d, torch.zeros_like(d))
            first = False
            px.copy_(x)
            py.copy_(y)
            steps += active.long()
            fl = v.state["flags"]
            fin = torch.where(active, (fl & 2) != 0, fin)
            crash = torch.where(active, (fl & 1) != 0, crash)
            prog = torch.where(active, info[:, 1], prog)
            speed = torch.where(active, info[:, 0], speed)
            active &= ~done.bool()
            if t % 50 == 49 and not bool(active.any()):
                break
        fin, crash = fin.cpu().numpy(), crash.cpu().numpy()
        prog, speed = prog.cpu().numpy(), speed.cpu().numpy()
        steps, total_reward, total_dist = steps.cpu().numpy(), total_reward.cpu().numpy(), total_dist.cpu().numpy()
        ok = fin
        eff = prog > 0.01
        res = {
            "num_episodes": int(N),
            "num_successful": int(ok.sum()),
            "success_rate": float(ok.mean()),
            "crash_rate": float(crash.mean()),
            "avg_steps": float(steps[ok].mean()) if ok.any() else 0,
            "avg_reward": float(total_reward[ok].mean()) if ok.any() else 0,
            "avg_progress": float(prog[ok].mean()) if ok.any() else 0,
            "avg_speed": float(speed[ok].mean()) if ok.any() else 0,
            "avg_distance": float(total_dist[ok].mean()) if ok.any() else 0,
            "avg_steps_per_progress": float((steps[eff] / prog[eff]).mean()) if eff.any() else float("nan"),
        }
        return res

    def close(self):
        self.venv.close()
