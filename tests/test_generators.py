"""CPU checks of the generator restatements the GPU generator tests rely on
(oracle/oracle.py; csrc/qpb_gen.hip is the product).

* glibc jump-ahead (glibc_draws_at) against the sequential glibc restatement,
  which tests/test_oracle.py pins to libc's own rand();
* Philox4x32-10 against the Random123 known-answer vectors (kat_vectors:
  philox4x32 10 rounds);
* the family restatement's structure (box rows, unit dense rows, shards).
"""
import numpy as np
import pytest

import oracle


@pytest.mark.parametrize("seed", [1, 42, 4001, 16001, 2**31 + 5])
def test_glibc_jump_ahead_matches_sequential(seed):
    g = oracle.GlibcRand(seed)
    seq = np.array([g.rand() for _ in range(3000)], dtype=np.float64)
    for first in (0, 1, 30, 31, 32, 288, 1000, 2500):
        assert np.array_equal(oracle.glibc_draws_at(seed, first, 300)[: len(seq[first:first + 300])],
                              seq[first:first + 300])


def test_ref_generate_at_matches_sequential_generator():
    P, q, x0 = oracle.ref_generate(16001, 5, 16)
    for k in range(5):
        Pk, qk, xk = oracle.ref_generate_at(16001, k, 16)
        assert np.array_equal(Pk, P[k]) and np.array_equal(qk, q[k]) and np.array_equal(xk, x0[k])


# Random123 kat_vectors, philox4x32 with 10 rounds: (ctr0..3, key0..1) -> out0..3
PHILOX_KAT = [
    ((0, 0, 0, 0, 0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 6, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("inp,out", PHILOX_KAT)
def test_philox_known_answers(inp, out):
    assert tuple(int(v) for v in oracle.philox4x32_10(*inp)) == out


def test_family_restatement_structure():
    H, f, A, b = oracle.family_generate(16, 6, 123, "box")
    assert np.allclose(H, np.transpose(H, (0, 2, 1)))
    assert np.all(np.linalg.eigvalsh(H) >= 1.0 - 1e-9)  # B^T B / (1e3 n) + I
    assert np.array_equal(A[0], np.concatenate([np.eye(16), -np.eye(16)])) and np.all(b == 10.0)
    assert np.all(np.abs(f) <= 1e3)
    H2, f2, A2, b2 = oracle.family_generate(16, 3, 123, "box", first=2)
    assert np.array_equal(f2, f[2:5]) and np.allclose(H2, H[2:5], rtol=0, atol=0)
    _, _, Ad, bd = oracle.family_generate(8, 4, 9, "dense")
    assert np.allclose(np.linalg.norm(Ad, axis=2), 1.0) and np.all((bd >= 1.0) & (bd < 10.0))
