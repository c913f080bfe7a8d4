"""Wire format: csrc/qpb_wire.c through the C-ABI,
against the restatements of the reference's writer (test/test.c:108-126 ->
oracle.write_wire) and reader (test/qp_ref.py:8-30 -> oracle.read_wire).
Host-only code: these run without a GPU (the library loads; no HIP call)."""
import os

import numpy as np
import pytest

import oracle

qpb = pytest.importorskip("qpb")


def _batch(B, n, m, seed=0):
    rng = np.random.default_rng(seed)
    H = rng.standard_normal((B, n, n))
    f = rng.standard_normal((B, n))
    A = rng.standard_normal((B, m, n)) if m else None
    b = rng.standard_normal((B, m)) if m else None
    return H, f, A, b


def test_single_qp_is_the_reference_format(tmp_path):
    H, f, _, _ = _batch(1, 5, 0)
    ours, ref = tmp_path / "ours.bin", tmp_path / "ref.bin"
    qpb.wire_write(str(ours), H, f)
    oracle.write_wire(str(ref), H[0], f[0])
    assert ours.read_bytes() == ref.read_bytes()  # byte-identical to test.c's writer
    n, P, q = oracle.read_wire(str(ours))          # and readable by qp_ref.py's reader
    assert n == 5 and np.array_equal(P, H[0]) and np.array_equal(q, f[0])
    H2, f2, A2, b2 = qpb.wire_read(str(ref))       # a test.c file read by the library
    assert np.array_equal(H2[0], H[0]) and np.array_equal(f2[0], f[0]) and A2.shape == (1, 0, 5)


@pytest.mark.parametrize("B,n,m", [(3, 4, 8), (1, 16, 32), (7, 16, 0), (2, 1, 3)])
def test_batched_round_trip(tmp_path, B, n, m):
    H, f, A, b = _batch(B, n, m, seed=B * 100 + n)
    path = str(tmp_path / "batch.bin")
    qpb.wire_write(path, H, f, A, b)
    assert os.path.getsize(path) == 8 * (3 + B * (n * n + n + m * n + m)) or (m == 0 and B == 1)
    H2, f2, A2, b2 = qpb.wire_read(path)
    assert np.array_equal(H2, H) and np.array_equal(f2, f)
    if m:
        assert np.array_equal(A2, A) and np.array_equal(b2, b)
    # the numpy restatement reads the same bytes
    H3, f3, A3, b3 = oracle.read_wire_batch(path)
    assert np.array_equal(H3, H) and np.array_equal(f3, f)
    # and writes the same bytes
    ref = str(tmp_path / "ref.bin")
    oracle.write_wire_batch(ref, H, f, A, b)
    assert open(ref, "rb").read() == open(path, "rb").read()


def test_bad_files_are_rejected(tmp_path):
    H, f, A, b = _batch(2, 4, 8)
    path = tmp_path / "x.bin"
    qpb.wire_write(str(path), H, f, A, b)
    data = path.read_bytes()
    (tmp_path / "trunc.bin").write_bytes(data[:-8])
    with pytest.raises(qpb.QPBError):
        qpb.wire_read(str(tmp_path / "trunc.bin"))
    (tmp_path / "badn.bin").write_bytes(np.array([2.5, 0.0, 1.0]).tobytes())
    with pytest.raises(qpb.QPBError):
        qpb.wire_read(str(tmp_path / "badn.bin"))
    with pytest.raises(qpb.QPBError):
        qpb.wire_read(str(tmp_path / "missing.bin"))


REF_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")


@pytest.mark.parametrize("n,seed", [(4, 7), (4, 20261015), (16, 1), (16, 99)])
def test_bytes_of_the_reference_writer(tmp_path, n, seed):
    """Pinned to the reference itself: oracle/_ref/wire_ref_n<N> runs the
    unmodified test_reference() (test/test.c:108-130) on a QP from the
    reference generator and keeps the file it writes (wire_driver.c).  Our
    writer must produce the same bytes and our reader must return its P, q."""
    import subprocess
    exe = os.path.join(REF_DIR, f"wire_ref_n{n}")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (make -C oracle ref, where /root/reference exists)")
    subprocess.run([exe, str(seed)], cwd=tmp_path, check=True, timeout=60)
    ref_bytes = (tmp_path / "wire_ref.bin").read_bytes()
    pq = np.frombuffer((tmp_path / "pq.bin").read_bytes(), dtype=np.float64)
    P, q = pq[: n * n].reshape(1, n, n), pq[n * n:].reshape(1, n)
    ours = tmp_path / "ours.bin"
    qpb.wire_write(str(ours), P, q)
    assert ours.read_bytes() == ref_bytes
    H2, f2, A2, b2 = qpb.wire_read(str(tmp_path / "wire_ref.bin"))
    assert np.array_equal(H2[0], P[0]) and np.array_equal(f2[0], q[0]) and A2.shape == (1, 0, n)
    nn, P3, q3 = oracle.read_wire(str(tmp_path / "wire_ref.bin"))  # qp_ref.py:8-30 restated
    assert nn == n and np.array_equal(P3, P[0]) and np.array_equal(q3, q[0])
