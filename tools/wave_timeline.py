#!/usr/bin/env python3
"""Wave timeline of the shipped n = 16 kernel at the metric's batch: where the
launch's time goes between the waves ("slot fill").

Needs the diagnostic build (the shipped gi_dense kernel plus two clock reads
and one 40-byte store per wave):

  VFLAGS=-DQPB_WAVE_TRACE tools/build_variant.sh \\
      embedded-qp-solver_amd/csrc/qpb_gi.hip wtrace
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_wtrace.so python tools/wave_timeline.py [B] [family]

Each wave records its start and end on the 100 MHz real-time counter and the
shader clock, and its hardware location (HW_ID, XCC_ID).  From those:
  - slot fill: the SIMDs' resident-wave time over 3 x the launch span (the
    kernel runs 3 waves per SIMD), split into ramp-up, steady state and tail;
  - the time a SIMD holds fewer than 3 waves while more waves are still to
    start (replacement gaps), and the gap from a wave's end to the start of
    the wave that takes its slot;
  - the shader clock each wave ran at, Δs_memtime / Δs_memrealtime x 100 MHz
    (MI355X_MICROARCH.md "DVFS give-back" item 6), unprofiled.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fam = sys.argv[2] if len(sys.argv) > 2 else "box"
OCC = 3
assert "wtrace" in qpb.LIB_PATH, "run with QPB_LIB=.../libqpb_wtrace.so (the QPB_WAVE_TRACE build)"
dev = torch.device("cuda", 0)
H, f, A, b = qpb.generate(16, B, 20261015, family=fam)
assert A.shape[1] == 32
waves = (B + 3) // 4
rec = torch.zeros(8 * waves, dtype=torch.int64, device=dev)  # 8 words per wave, see qpb_gi.hip
sol = qpb.solve(H, f, A, b)
for _ in range(3):  # warm: the clock settles under back-to-back launches
    qpb.solve(H, f, A, b, out=sol)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
plain = []
for _ in range(10):
    e0.record()
    qpb.solve(H, f, A, b, out=sol)
    e1.record()
    torch.cuda.synchronize()
    plain.append(e0.elapsed_time(e1))


def traced():
    # the C entry point directly: qpb.solve_sections would pass its own
    # 256 x 20 buffer, and this build writes 8 words per wave
    d = qpb.Desc(16, 32, B, 0, 0, 0.0)
    rc = qpb._lib.qpb_solve_sections(ctypes.byref(d), qpb._ptr(H), qpb._ptr(f), qpb._ptr(A), qpb._ptr(b),
                                     qpb._ptr(sol.x), qpb._ptr(sol.lam), qpb._ptr(sol.active),
                                     qpb._ptr(sol.status), qpb._ptr(sol.iters), qpb._ptr(rec), rec.numel(),
                                     qpb._stream_ptr(None))
    qpb._check(rc, "qpb_solve_sections (wave trace)")


traced()
torch.cuda.synchronize()
rec.zero_()
e0.record()
traced()
e1.record()
torch.cuda.synchronize()
traced_ms = e0.elapsed_time(e1)
r = rec.view(waves, 8).cpu().numpy().view(np.uint64)
assert (r[:, 1] > 0).all(), "every wave wrote its record"

rt0 = r[:, 0].astype(np.int64)
rt1 = r[:, 1].astype(np.int64)
rtl = r[:, 5].astype(np.int64)  # the inputs have arrived
mt = (r[:, 3] - r[:, 2]).astype(np.float64)
hw = (r[:, 4] & np.uint64(0xFFFFFFFF)).astype(np.int64)
xcc = (r[:, 4] >> np.uint64(32)).astype(np.int64) & 0xF
t0 = rt0.min()
s = (rt0 - t0) * 10.0 / 1000.0  # us
e = (rt1 - t0) * 10.0 / 1000.0
life = e - s
span = e.max()
# HW_ID (gfx9): wave_id 3:0, simd_id 5:4, pipe 7:6, cu_id 11:8, sh_id 12, se_id 15:13
simd_key = xcc * (1 << 16) + (((hw >> 13) & 7) << 8) + (((hw >> 12) & 1) << 7) + (((hw >> 8) & 0xF) << 2) + ((hw >> 4) & 3)
keys, inv, per_simd = np.unique(simd_key, return_inverse=True, return_counts=True)
nsimd = len(keys)
cus = len(np.unique(simd_key >> 2))

# time-weighted resident-wave count per SIMD, split by phase
ramp_t = np.zeros(nsimd)   # before the SIMD first holds OCC waves
tail_t = np.zeros(nsimd)   # after the SIMD's last wave started
fill = {k: 0.0 for k in range(OCC + 2)}
fill_steady = {k: 0.0 for k in range(OCC + 2)}
gaps = []
order = np.lexsort((s, inv))
starts_by = np.split(order, np.cumsum(per_simd)[:-1])
short_steady = 0.0
for k, idx in enumerate(starts_by):
    ss, ee = s[idx], e[idx]
    ev_t = np.concatenate([ss, ee])
    ev_d = np.concatenate([np.ones_like(ss), -np.ones_like(ee)])
    o = np.lexsort((ev_d, ev_t))  # ends before starts at equal times
    ev_t, ev_d = ev_t[o], ev_d[o]
    c = np.cumsum(ev_d)
    dt = np.diff(np.concatenate([[0.0], ev_t, [span]]))
    cc = np.concatenate([[0], c])
    last_start = ss.max()
    first_full = ev_t[np.argmax(c >= OCC)] if (c >= OCC).any() else last_start
    tt = np.concatenate([[0.0], ev_t])
    for ci, d, ti in zip(cc, dt, tt):
        fill[min(int(ci), OCC + 1)] += d
        if first_full <= ti < last_start:
            fill_steady[min(int(ci), OCC + 1)] += d
            if ci < OCC:
                short_steady += d
    ramp_t[k] = first_full
    tail_t[k] = span - last_start
    # slot hand-over gaps: the i-th start after the first OCC takes the slot of
    # the (i - OCC + 1)-th end in end order (a FIFO pool of OCC slots)
    ends_sorted = np.sort(ee)
    for i in range(OCC, len(ss)):
        gaps.append(ss[i] - ends_sorted[i - OCC])
gaps = np.array(gaps)


def concurrency(key):
    """time share of each resident-wave count over the units `key` names
    (CUs, SIMDs), and each unit's maximum"""
    ks, iv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    share = {}
    mx = []
    for idx in np.split(np.lexsort((s, iv)), np.cumsum(cnt)[:-1]):
        ev_t = np.concatenate([s[idx], e[idx]])
        ev_d = np.concatenate([np.ones(len(idx)), -np.ones(len(idx))])
        o = np.lexsort((ev_d, ev_t))
        ev_t, ev_d = ev_t[o], ev_d[o]
        c = np.cumsum(ev_d).astype(int)
        dt = np.diff(np.concatenate([ev_t, [span]]))
        for ci in np.unique(c):
            share[int(ci)] = share.get(int(ci), 0.0) + float(dt[c == ci].sum())
        mx.append(int(c.max()))
    tot_t = len(ks) * span
    return ({str(k): round(v / tot_t, 4) for k, v in sorted(share.items())},
            {str(v): int(n) for v, n in zip(*np.unique(mx, return_counts=True))})


cu_share, cu_max = concurrency(simd_key >> 2)
simd_share, simd_max = concurrency(simd_key)
tot = nsimd * span
clock = mt / ((rt1 - rt0) * 10e-9) / 1e9  # GHz
resident = life.sum() / (OCC * nsimd * span)

out = {
    "B": B,
    "family": fam,
    "library": qpb.version(),
    "waves": waves,
    "simds_seen": int(nsimd),
    "cus_seen": int(cus),
    "xcds_seen": int(len(np.unique(xcc))),
    "waves_per_simd": {"min": int(per_simd.min()), "max": int(per_simd.max()), "mean": float(per_simd.mean())},
    "plain_kernel_ms_median": float(np.median(plain)),
    "traced_kernel_ms": traced_ms,
    "span_us": float(span),
    "wave_lifetime_us": {"mean": float(life.mean()), "p50": float(np.median(life)),
                         "p99": float(np.percentile(life, 99)), "max": float(life.max())},
    "input_wait_us": {"mean": float(((rtl - rt0) * 0.01).mean()), "p50": float(np.median((rtl - rt0) * 0.01)),
                      "p90": float(np.percentile((rtl - rt0) * 0.01, 90))},
    "end_after_store_drain": "wtrace2" in qpb.LIB_PATH,
    "slot_fill": float(resident),
    "time_share_by_resident_waves": {str(k): round(v / tot, 4) for k, v in fill.items()},
    "cu_time_share_by_resident_waves": cu_share,
    "cu_max_resident_waves": cu_max,
    "simd_max_resident_waves": simd_max,
    "steady_state_share_below_occ": round(short_steady / max(1e-9, sum(fill_steady.values())), 4),
    "ramp_us_mean": float(ramp_t.mean()),
    "tail_us": {"mean": float(tail_t.mean()), "max": float(tail_t.max()), "min": float(tail_t.min())},
    "slot_handover_gap_us": {"mean": float(gaps.mean()), "p50": float(np.median(gaps)),
                             "p90": float(np.percentile(gaps, 90)), "p99": float(np.percentile(gaps, 99))},
    "first_start_us_by_xcd": [float(s[xcc == x].min()) for x in range(8)],
    "last_end_us_by_xcd": [float(e[xcc == x].max()) for x in range(8)],
    "shader_clock_GHz": {"p10": float(np.percentile(clock, 10)), "p50": float(np.median(clock)),
                         "p90": float(np.percentile(clock, 90))},
}
# the shader clock the waves ran at, by their start time (100 us bins): does
# the chip raise its clock during a launch?
cb = (s // 100).astype(int)
out["shader_clock_GHz_by_start_100us"] = [round(float(np.median(clock[cb == i])), 3) if (cb == i).any() else None
                                          for i in range(int(cb.max()) + 1)]
# chip-level resident waves in 10 us bins (the shape of ramp and tail)
bins = np.arange(0.0, span + 10.0, 10.0)
occ = np.zeros(len(bins) - 1)
for lo, hi in zip(s, e):
    i0, i1 = int(lo // 10), int(hi // 10)
    occ[i0:i1 + 1] += 1  # coarse: counts a wave in every bin it touches
out["resident_waves_per_10us_bin"] = occ.astype(int).tolist()
od = os.path.join(ROOT, "gpurun_out", "wtrace")
os.makedirs(od, exist_ok=True)
tag = "_drain" if "wtrace2" in qpb.LIB_PATH else ""
with open(os.path.join(od, f"wave_timeline_{fam}_{B}{tag}.json"), "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps({k: v for k, v in out.items() if k not in ("resident_waves_per_10us_bin", "library")}, indent=1))
