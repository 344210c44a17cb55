"""Batched evaluation -- evaluate.py:12-122,173-238 and utils/metrics.py:39-142.

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
            st = v.state  # writes the stepped state back into x, y, flags (rx_state_export)
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
            fl = st["flags"]
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
            "all_episodes": _episodes(total_reward, steps, prog, fin, crash, speed, total_dist),
        }
        return res

    def close(self):
        self.venv.close()


def _episodes(total_reward, steps, prog, fin, crash, speed, dist, placement=None):
    """Per-episode dicts (utils/metrics.py:70-78 / 131-141 keys), evaluate.py's 'all_episodes'."""
    out = []
    for i in range(len(steps)):
        n = int(steps[i])
        m = {"total_reward": float(total_reward[i]), "steps": n, "progress": float(prog[i]),
             "finished": bool(fin[i]), "crashed": bool(crash[i]), "speed": float(speed[i]),
             "total_distance": float(dist[i]), "distance_per_step": float(dist[i]) / n if n > 1 else 0.0}
        if placement is not None:
            m["placement"] = int(placement[i]) if placement[i] > 0 else None
        out.append(m)
    return out


class MultiEvaluator:
    """evaluate.py:68-122 + utils/metrics.py:80-142 (self-play model): every
    two-car episode of the protocol at once, BOTH cars driven by the evaluated
    policy (one batched forward over the 2N car observations per step), at
    most 3,000 steps, stopping at dones['__all__'].  The reported agent is car
    0 unless only car 1 finished (metrics.py:124-131)."""

    def __init__(self, num_tracks=40, num_runs=5, seed=42, global_seed=0, max_steps=3000, device=None,
                 n_sensors=11, env_seed=0):
        from .vector_env import RacingVectorEnv
        cps, ws, self.ids = eval_pool(num_tracks, num_runs, seed, global_seed)
        self.max_steps = max_steps
        self.venv = RacingVectorEnv(cps, ws, n_agents=2, n_sensors=n_sensors, device=device, autoreset="disabled",
                                    seed=env_seed)
        self.device = self.venv.device

    @torch.no_grad()
    def run(self, agent):
        v = self.venv
        N, D = v.num_envs, v.D
        dev = self.device
        obs = v.reset_device()
        active = torch.ones(N, dtype=torch.bool, device=dev)
        total_reward = torch.zeros((N, 2), dtype=torch.float64, device=dev)
        total_dist = torch.zeros((N, 2), dtype=torch.float64, device=dev)
        steps = torch.zeros(N, dtype=torch.int64, device=dev)
        info_last = torch.zeros((N, 2, 4), dtype=torch.float64, device=dev)
        flags_last = torch.zeros((N, 2), dtype=torch.uint8, device=dev)
        x, y = v.state["x"].view(N, 2), v.state["y"].view(N, 2)
        px, py = x.clone(), y.clone()
        first = True
        for t in range(self.max_steps):
            a = agent.get_action_and_value(obs.reshape(2 * N, D))[0].reshape(N, 2, 2)
            obs, _, done = v.step_device(a, full_info=True)
            st = v.state  # writes the stepped state back into x, y, flags (rx_state_export)
            act2 = active.unsqueeze(1)
            total_reward += torch.where(act2, v.buf["reward64"], torch.zeros_like(total_reward))
            if not first:
                d = torch.sqrt((x - px) ** 2 + (y - py) ** 2)
                total_dist += torch.where(act2, d, torch.zeros_like(d))
            first = False
            px.copy_(x)
            py.copy_(y)
            steps += active.long()
            info_last = torch.where(act2.unsqueeze(2), v.buf["info"], info_last)
            flags_last = torch.where(act2, st["flags"].view(N, 2), flags_last)
            active &= ~done.bool()
            if t % 50 == 49 and not bool(active.any()):
                break
        fin = (flags_last & 2) != 0
        crash = (flags_last & 1) != 0
        pick = (~fin[:, 0] & fin[:, 1]).long()  # car 1 only if it finished and car 0 did not
        ar = torch.arange(N, device=dev)
        g = lambda t: t[ar, pick].cpu().numpy()  # noqa: E731
        fin_c, crash_c = g(fin), g(crash)
        prog, speed, place = g(info_last[:, :, 1]), g(info_last[:, :, 0]), g(info_last[:, :, 3])
        rew, dist = g(total_reward), g(total_dist)
        steps = steps.cpu().numpy()
        ok = fin_c
        eff = prog > 0.01
        return {
            "num_episodes": int(N),
            "num_successful": int(ok.sum()),
            "success_rate": float(ok.mean()),
            "crash_rate": float(crash_c.mean()),
            "avg_steps": float(steps[ok].mean()) if ok.any() else 0,
            "avg_reward": float(rew[ok].mean()) if ok.any() else 0,
            "avg_progress": float(prog[ok].mean()) if ok.any() else 0,
            "avg_speed": float(speed[ok].mean()) if ok.any() else 0,
            "avg_distance": float(dist[ok].mean()) if ok.any() else 0,
            "avg_steps_per_progress": float((steps[eff] / prog[eff]).mean()) if eff.any() else float("nan"),
            "all_episodes": _episodes(rew, steps, prog, fin_c, crash_c, speed, dist, place),
        }

    def close(self):
        self.venv.close()
