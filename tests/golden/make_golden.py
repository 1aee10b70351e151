"""Generates the committed golden vectors of tests/test_oracle.py from the oracle.

Run from the repo root: python tests/golden/make_golden.py
The vectors pin the CPU restatement against regressions (they are not
reference outputs: Mitsuba is not installed here).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def make(name, N, A, regular, spp, seed):
    cfg = benchy_index_matched(N=N, angles=A, regular_sampling=regular, spp=spp)
    d = desc_from_config(cfg)
    rng = np.random.default_rng(1234)
    pat = rng.uniform(0.0, 0.1, A * N * N).astype(np.float32)
    G = rng.uniform(-1.0, 1.0, (N, N, N)).astype(np.float32)
    dose, visits = oracle.forward(d, pat, spp=spp, seed=seed)
    grad, _ = oracle.adjoint(d, G, spp=spp, seed=seed)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), N=N, A=A, regular=regular, spp=spp, seed=seed,
                        patterns=pat, grad_dose=G, dose=dose, grad=grad, visits=visits)
    print(name, visits, float(dose.sum()))


if __name__ == "__main__":
    oracle.build()
    make("im16_a8_regular", 16, 8, True, 1, 0)
    make("im16_a8_jitter_spp2", 16, 8, False, 2, 7)
