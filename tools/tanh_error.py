"""Float32 emulation of rx_policy::tanh_fast (csrc/rx_policy.h): the exp form
sign(x) (1 - 2 / (exp2(2|x| log2 e) + 1)) with correctly rounded exp2 and
reciprocal, against float64 tanh -- the error bound the header states."""
import numpy as np

x = np.linspace(-12, 12, 2_000_001).astype(np.float32)
x = np.concatenate([x, (np.random.default_rng(0).standard_normal(1_000_000) * 0.05).astype(np.float32)])
ref = np.tanh(x.astype(np.float64))
e = np.exp2(np.abs(x) * np.float32(2.8853900817779268)).astype(np.float32)
r = (np.float32(1) / (e + np.float32(1))).astype(np.float32)
y = np.copysign((np.float32(1) - np.float32(2) * r).astype(np.float32), x)
err = np.abs(y - ref)
print(f"max abs error {err.max():.3g} (float32 tanh itself: {np.abs(np.tanh(x).astype(np.float64) - ref).max():.3g})")
