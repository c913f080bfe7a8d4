"""Host logic of bench.py (CPU, no GPU): the algorithmic bytes per QP behind
the roofline, the BASELINE config naming, the committed PMC
lookup (keyed by the hot kernel's revision inside the library version string)
and the VALU issue-rate ceiling computed from it."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # module level imports only the stdlib
    return mod


def test_bytes_per_qp_metric_config(bench):
    # n = 16, m = 32: H 2048 + f 128 + A 4096 + b 256 in, x 128 + lam 256 + mask 4 + status 4 out
    assert bench.bytes_per_qp(16, 32) == 6920
    assert bench.bytes_per_qp(32, 64) == 8 * (1024 + 32 + 2048 + 64) + 8 * 96 + 8 + 4
    assert bench.bytes_per_qp(128, 256) == 8 * (16384 + 128 + 32768 + 256) + 8 * 384 + 32 + 4


def test_baseline_config_names(bench):
    assert "configs[2]" in bench.baseline_config(16, 1 << 20, 8)
    assert "configs[1]" in bench.baseline_config(16, 65536, 1)
    assert "configs[4]" in bench.baseline_config(32, 262144, 1)
    assert "configs[3]" in bench.baseline_config(128, 16384, 1)
    assert bench.baseline_config(16, 1000, 1) == "not a BASELINE config"


def test_pmc_traffic_is_keyed_by_kernel_revision(bench):
    t = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    c = t["config"]
    lib_ok = "qpb x.y (gfx950; " + t["kernel_rev"] + ": desc, more; gi_box v1: ...)"
    got = bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"], c["family"], lib_ok)
    assert got is not None and got["bytes"] == t["hbm_bytes_per_launch"]
    assert got["valu_classes"] == t["valu_classes"]
    # another revision of the hot kernel, or another configuration: no number
    assert bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"], c["family"], "qpb (gi_dense v0)") is None
    # a revision that merely extends the committed one's name is another revision
    longer = "qpb x.y (gfx950; " + t["kernel_rev"] + ".1: desc)"
    assert bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"], c["family"], longer) is None
    assert bench.kernel_revisions(lib_ok) == {t["kernel_rev"], "gi_box v1"}
    assert bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"] // 2, c["family"], lib_ok) is None
    assert bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"], "dense", lib_ok) is None


def test_valu_ceiling(bench):
    assert bench.valu_ceiling(None, 1, 1.0) is None
    t = {"valu_classes": {"VALU": 3000.0, "FMA_F64": 1000.0, "MUL_F64": 300.0, "ADD_F64": 100.0,
                          "TRANS_F64": 40.0}, "valu_source": "x"}
    waves = 1 << 18  # 1 M QPs, four per wave
    v = bench.valu_ceiling(t, waves, 2.0)
    c = bench.VALU_COST
    cyc = 1000 * c["FMA_F64"] + 300 * c["MUL_F64"] + 100 * c["ADD_F64"] + 40 * c["TRANS_F64"] + 1560 * c["B32"]
    # every class at its measured cost, 256 waves per SIMD at 2.4 GHz
    assert v["issue_cycles_per_wave"] == pytest.approx(cyc)
    assert v["ceiling_ms"] == pytest.approx(cyc * 256 / 2.4e9 * 1e3)
    assert v["frac"] == pytest.approx(v["ceiling_ms"] / 2.0)
    assert v["classes_per_wave"]["B32"] == pytest.approx(1560.0)


def test_committed_pmc_matches_the_built_library(bench):
    # the bench line's roofline.traffic and valu_ceiling come from the committed
    # PMC file only while it names the hot kernel revision the in-tree library
    # reports; a kernel change without a new PMC pass must show up here
    import sys
    sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
    import qpb
    t = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    c = t["config"]
    assert bench.pmc_traffic(c["n"], c["m"], c["batch_per_gpu"], c["family"], qpb.version()) is not None


def test_cpu_run_refuses_to_fork_after_gpu_init(bench, monkeypatch):
    """bench.cpu_run forks one worker per CPU; after this process has
    initialised the GPU the workers would inherit the HIP runtime (round 3's
    config-sweep SIGSEGV), so it must refuse instead of forking."""
    import sys
    import types
    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(is_initialized=lambda: True))
    monkeypatch.setitem(sys.modules, "torch", fake)
    with pytest.raises(RuntimeError, match="initialised"):
        bench.cpu_run("ref_admm_batch", 1, [[0.0]], [0.0], 0.1, 1)


def test_cpu_run_before_gpu_init_is_allowed(bench, monkeypatch):
    import sys
    import types
    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(is_initialized=lambda: False))
    monkeypatch.setitem(sys.modules, "torch", fake)
    # no reference library under this name: returns None without forking
    assert bench.cpu_run("ref_admm_batch", 1, [[0.0]], [0.0], 0.1, 1, lib_name="absent.so") is None


def test_shard_prediction_is_keyed_by_kernel_revision(bench):
    # the N > 1 line's kernel-bound speed-up comes from the committed batch
    # scan only while the scan names a hot-kernel revision of the loaded
    # library: a stale scan yields no prediction
    scan = json.load(open(os.path.join(ROOT, "profiles", "batch_scan.json")))
    rev = scan["revision"]
    lib_ok = "qpb x.y (gfx950; " + rev + ": desc; gi_box v1: ...)"
    got = bench.shard_time_prediction(16, 32, "box", 131072, 1048576, lib_ok)
    assert got is not None and got["revision"] == rev
    assert got["kernel_bound_speedup"] == pytest.approx(got["total_kernel_ms"] / got["shard_kernel_ms"])
    assert bench.shard_time_prediction(16, 32, "box", 131072, 1048576, "qpb (gi_dense v0: x)") is None
    assert bench.shard_time_prediction(16, 32, "dense", 131072, 1048576, lib_ok) is None
