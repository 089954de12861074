"""The device retainBest permutation's formulation (k_select_stl in csrc/orb.hip) against the C++
standard library it restates, on the CPU.

tests/cpp/stl_select_model.cpp restates the device algorithm (one parallel pass per Hoare
partition: the k-th left stopper swaps with the k-th right stopper, K = max_x min(#L before x,
#R at or after x), cut = min(L[K], R[K-1])), asserts on every pass that the device's K-free rules
(an L of rank ra is swapped iff ra + rb + isR < nR, an R iff ra + rb >= nR; the cut is the first
unswapped L or swapped R) pick the same swaps and cut, and compares its permutation with std::nth_element +
std::partition (OpenCV KeyPointsFilter::retainBest) on random, tie-heavy,
sorted and McIlroy-adversarial inputs — the latter drive libstdc++ into its heap-select fallback.
"""
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def test_device_formulation_equals_libstdcxx(tmp_path):
    exe = tmp_path / "stl_select_model"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "cpp", "stl_select_model.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all identical" in r.stdout and "heap select exercised" in r.stdout


def test_oracle_retain_best_keys_semantics(oracle):
    """orc_retain_best_keys keeps exactly {key >= the npts-th largest} (ties included), first
    npts entries hold the npts largest."""
    rng = np.random.default_rng(5)
    for n, npts, hi in [(1, 1, 3), (10, 3, 2), (500, 100, 7), (2000, 868, 255), (3000, 1, 1 << 30)]:
        keys = rng.integers(0, hi, n).astype(np.uint32)
        idx = oracle.retain_best_keys(keys, npts)
        if n <= npts:
            assert list(idx) == list(range(n))
            continue
        kth = np.sort(keys)[::-1][npts - 1]
        assert sorted(idx) == sorted(np.nonzero(keys >= kth)[0])
        assert keys[idx[:npts]].min() >= kth and keys[idx[npts - 1]] == kth


def test_antiqsort_keys(oracle):
    keys = oracle.antiqsort(1000, 499)
    assert len(keys) == 1000 and keys.max() <= 999
    assert len(oracle.retain_best_keys(keys, 500)) >= 500
