"""Exactness of the arithmetic rewrites the HIP kernel makes relative to the
reference's literal expressions (each must be bit-identical, since the GPU
results are compared bit-for-bit with the oracle), and accuracy of the
transcendental sequence shared by oracle and kernel."""
import numpy as np
import pytest

F = np.float32


def test_rejection_test_without_sqrt_is_exact():
    """length(r) > 1 (Main.cu:197) <=> RN(x*x+y*y+z*z) > 1 + 2^-23, for every
    float s in [0.25, 4) (outside it both sides are trivially equal)."""
    one_ulp = F(1.00000012)
    assert one_ulp.view(np.uint32) == F(1).view(np.uint32) + 1
    lo, hi = F(0.25).view(np.uint32), F(4.0).view(np.uint32)
    for start in range(int(lo), int(hi), 1 << 24):
        s = np.arange(start, min(start + (1 << 24), int(hi)), dtype=np.uint32).view(np.float32)
        assert np.array_equal(np.sqrt(s) > F(1), s > one_ulp)


def test_rand_range_rewrite_is_exact():
    """float(u)/INT_MAX*0.5f*max (Math.cuh:278) == float(u) * (2^-32 * max)."""
    rng = np.random.default_rng(1)
    u = np.concatenate([rng.integers(0, 2**32, 200000, dtype=np.uint64),
                        np.array([0, 1, 2**31, 2**32 - 1, 2**32 - 128, 2**32 - 129], dtype=np.uint64)])
    fu = u.astype(np.float32)
    for mx in (F(1), F(2)):
        ref = ((fu / F(2147483648.0)) * F(0.5)) * mx
        new = fu * (F(2.3283064365386963e-10) * mx)
        assert np.array_equal(ref.view(np.uint32), new.view(np.uint32))


def test_sphere_early_out_is_exact():
    """b >= 0, finite disc >= 0, a2 > 0  =>  t = (-b - sqrt(disc)) / a2 <= 1e-4:
    the reference rejects such hits, so the kernel may skip sqrt/div."""
    rng = np.random.default_rng(2)
    b = np.abs(rng.standard_normal(100000).astype(F)) * F(10)
    disc = np.abs(rng.standard_normal(100000).astype(F)) * F(100)
    a2 = (np.abs(rng.standard_normal(100000).astype(F)) + F(0.5)) * F(2)
    t = (-b - np.sqrt(disc)) / a2
    assert (t <= F(1e-4)).all()


def _ulp_err(got, want):
    want32 = np.float32(want)
    spacing = np.abs(np.spacing(want32)).astype(np.float64)
    return np.abs(got.astype(np.float64) - want) / np.maximum(spacing, 1e-45)


@pytest.mark.parametrize("fn,ref,lo,hi,maxulp", [
    ("orc_sinf", np.sin, 0.0, 2 * np.pi, 4.0),
    ("orc_cosf", np.cos, 0.0, 2 * np.pi, 4.0),
    ("orc_atanf", np.arctan, 0.0, 50.0, 4.0),
])
def test_transcendental_accuracy(oracle, fn, ref, lo, hi, maxulp):
    """The Cody-Waite + minimax sequence (oracle.c, rt_kernels.hip) against
    float64 libm over the arguments the path uses (phi = 2*pi*e2 in [0, 2pi],
    theta in [0, pi/2], atan of [0, inf))."""
    f = getattr(oracle.lib(), fn)
    xs = np.linspace(lo, hi, 4001, dtype=np.float32)
    got = np.array([f(float(x)) for x in xs], dtype=np.float32)
    want = ref(xs.astype(np.float64))
    big = np.abs(want) > 1e-3
    assert _ulp_err(got[big], want[big]).max() <= maxulp
    assert np.abs(got.astype(np.float64) - want).max() < 4e-7


def test_atan_of_infinity(oracle):
    assert abs(oracle.lib().orc_atanf(float("inf")) - np.pi / 2) < 1e-7
    assert oracle.lib().orc_atanf(0.0) == 0.0


@pytest.mark.gpu
def test_sqrt_rcp_helpers_exhaustive():
    """csrc/rt_sqrt.h's short in-range paths (sqrt_cr, rcp_cr, inv_length_cr)
    equal the compiler's correctly rounded sqrtf, 1/x and 1/sqrtf for every
    one of the 2^32 float inputs (tools/sqrt_exhaustive.hip on the GPU,
    built by __graft_entry__.build())."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "sqrtx")
    assert os.path.exists(exe), "build/sqrtx missing: run __graft_entry__.build()"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "inputs evaluated: 4294967296 of 4294967296" in r.stdout, r.stdout
    assert r.stdout.count(": 0 mismatches") == 3, r.stdout
