"""The n <= 16 kernel's dynamic tail (qpb_gi.hip claim_tail_group): from
65 536 four-QP groups on, the last groups of a launch are claimed through
per-XCD counters instead of taken by workgroup index.

Every QP of such a launch must be solved exactly once and exactly as in a
launch without the tail: the outputs are pre-filled with sentinels (a group
that no workgroup claims keeps them), the batch is ragged (its last group
short, its ranges uneven), the launch is repeated on the same stream (the
counters are zeroed before each launch) and alternated over two streams, and
every output is compared bit for bit with the same QPs solved in slices of
65 532 QPs, below the tail's threshold.
"""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TAIL_MIN_QPS = 4 * 65536


@pytest.fixture(scope="module")
def qpb():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import qpb as q
    return q


def sentinel_out(qpb, B, n, m, dev):
    return qpb.Solution(torch.full((B, n), float("nan"), dtype=torch.float64, device=dev),
                        torch.full((B, m), float("nan"), dtype=torch.float64, device=dev),
                        torch.full((B, (m + 31) // 32), -1, dtype=torch.int32, device=dev),
                        torch.full((B,), -77, dtype=torch.int32, device=dev),
                        torch.full((B,), -77, dtype=torch.int32, device=dev))


def sliced(qpb, H, f, A, b, step=65532):
    parts = [qpb.solve(H[i:i + step].contiguous(), f[i:i + step].contiguous(), A[i:i + step].contiguous(),
                       b[i:i + step].contiguous()) for i in range(0, H.shape[0], step)]
    return qpb.Solution(*(torch.cat([p[k] for p in parts]) for k in range(5)))


def same(a, b):
    for k in range(5):
        x, y = a[k], b[k]
        if x.dtype == torch.float64:
            x, y = x.view(torch.int64), y.view(torch.int64)
        assert torch.equal(x, y), k


@pytest.mark.parametrize("B,family,m", [(TAIL_MIN_QPS + 4 * 8 * 37 + 3, "dense", 32), (TAIL_MIN_QPS, "box", 32),
                                        (TAIL_MIN_QPS + 1, "dense", 20), (TAIL_MIN_QPS + 6, "box", 16)])
def test_tail_claims_every_group_once(qpb, B, family, m):
    dev = torch.device("cuda", 0)
    H, f, A, b = qpb.generate(16, B, 777 + B, family=family, shift=1.0, box=10.0)
    if m != A.shape[1]:  # a ragged row count: the first m rows
        A, b = A[:, :m].contiguous(), b[:, :m].contiguous()
    ref = sliced(qpb, H, f, A, b)
    torch.cuda.synchronize()
    assert bool((ref.status == qpb.OK).all())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(3):
        st = (torch.cuda.current_stream(), s1, s2)[rep]
        with torch.cuda.stream(st):
            out = sentinel_out(qpb, B, 16, m, dev)
            got = qpb.solve(H, f, A, b, out=out)
        torch.cuda.synchronize()
        same(got, ref)
    for st in (s1, s2):  # the cached workspaces, before the streams go
        qpb.release_stream_workspace(st)
