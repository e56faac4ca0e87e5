"""Zig std.rand known-answer vectors (the RNG the reference's renderWorker
uses: std.rand.DefaultPrng = Xoshiro256, seeded through SplitMix64,
stage3.zig:225).  The zig submodule/toolchain is absent, so these are the
published test vectors of Zig 0.11's lib/std/rand/Xoshiro256.zig
("xoroshiro sequence", init(0)) and lib/std/rand/SplitMix64.zig
("splitmix64 sequence"), restated here as data."""
import numpy as np


def test_xoshiro256_sequence(oracle_mod):
    exp = [0x53175d61490b23df, 0x61da6f3dc380d507, 0x5c0fdf91ec9a7bfc,
           0x02eebf8c3bbe5e1a, 0x7eca04ebaf4a5eea, 0x0543c37757f08d9a]
    assert [int(x) for x in oracle_mod.xoshiro_u64(0, 6)] == exp


def test_splitmix64_sequence(oracle_mod):
    exp = [0x5dbd39db0178eb44, 0xa9900fb66b397da3, 0x5c1a28b1aeebcf5c,
           0x64a963238f776912, 0xc6d4177b21d1c0ab, 0xb2cbdbdb5ea35394]
    assert [int(x) for x in oracle_mod.splitmix_u64(0xaeecf86f7878dd75, 6)] == exp


def test_float_f32_in_unit_interval_and_distribution(oracle_mod):
    # Random.float(f32): [0, 1), mean 1/2, every value a multiple of 2^-24 or finer
    for f in (oracle_mod.xoshiro_f32(1, 200000), oracle_mod.path_f32(0, 5, 7, 200000)):
        assert (f >= 0).all() and (f < 1).all()
        assert abs(f.mean() - 0.5) < 0.005
        assert abs((f < 0.25).mean() - 0.25) < 0.005


def test_float_norm_moments(oracle_mod):
    # floatNorm(f32) via the NormDist ziggurat: N(0, 1)
    for z in (oracle_mod.xoshiro_norm(3, 400000), oracle_mod.path_norm(0, 1, 2, 400000)):
        assert abs(z.mean()) < 0.01
        assert abs(z.std() - 1.0) < 0.01
        assert abs((np.abs(z) < 1.0).mean() - 0.682689) < 0.004
        assert (np.abs(z) > 3.6541528853610088).any()    # tail (zero_case) reached


def test_ziggurat_tables(oracle_mod):
    x, f = oracle_mod.zig_tables()
    assert x[1] == 3.6541528853610088 and x[256] == 0.0
    assert np.all(np.diff(x[1:]) < 0)                      # strictly decreasing
    assert np.allclose(f, np.exp(-x * x / 2), rtol=1e-15, atol=0)
