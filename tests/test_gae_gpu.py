"""GAE kernels vs PPO.compute_advantages golden vectors (agent/ppo.py:134-154)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(g, tag, scan):
    from rx.gae import compute_gae
    c = lambda k: torch.from_numpy(g[f"{tag}_{k}"]).cuda()  # noqa: E731
    return compute_gae(c("rewards"), c("dones"), c("values"), c("next_value"), c("next_done"),
                       float(g[f"{tag}_gamma"]), float(g[f"{tag}_lambda"]), scan=scan)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_gae_bit_exact(golden, tag):
    g = golden["gae"]
    adv, ret = _run(g, tag, scan=False)
    assert np.array_equal(adv.cpu().numpy(), g[f"{tag}_adv"])
    assert np.array_equal(ret.cpu().numpy(), g[f"{tag}_ret"])


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_gae_scan_within_tolerance(golden, tag):
    """Affine-scan variant: different association, so equal to ~1e-6 relative."""
    g = golden["gae"]
    adv, ret = _run(g, tag, scan=True)
    ref = g[f"{tag}_adv"]
    scale = np.abs(ref).max()
    err = np.abs(adv.cpu().numpy() - ref).max()
    print(f"\nscan GAE [{tag}] max abs err {err:.3g} (max |A| {scale:.3g})")
    assert err <= 1e-5 * scale
    assert np.abs(ret.cpu().numpy() - g[f"{tag}_ret"]).max() <= 1e-5 * scale


def test_gae_large_vs_oracle(oracle):
    T, N = 128, 65536
    rng = np.random.default_rng(0)
    r = rng.normal(0, 10, (T, N)).astype(np.float32)
    v = rng.normal(0, 30, (T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.02).astype(np.float32)
    nv = rng.normal(0, 30, N).astype(np.float32)
    nd = rng.random(N) < 0.02
    from rx.gae import compute_gae
    adv, ret = compute_gae(*(torch.from_numpy(x).cuda() for x in (r, d, v, nv, nd)), 0.99, 0.95)
    oa, orr = oracle.gae(r, v, d, nv, nd, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), oa) and np.array_equal(ret.cpu().numpy(), orr)
