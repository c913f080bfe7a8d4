// qpb_common.h -- CDNA4 (gfx950) device helpers shared by the qpb kernels.
//
// The small-QP kernels map one QP onto one 16-lane DPP *row* of a 64-lane
// wavefront (4 QPs per wave).  Lane l of a row owns index l of every
// n-vector; cross-lane traffic inside a QP uses the gfx950 DPP row ops:
//   row_newbcast:J  (v_mov_b64_dpp, one instruction per double) -- lane J of
//                   the row broadcast to the whole row
//   row_ror:N       rotations for exact min/argmin all-reduces
// Every value that steers control flow is computed identically on all 16
// lanes of a row (broadcasts, exact min-reductions, replicated arithmetic),
// so a QP's lanes never diverge from each other.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <utility>

// Cached per-(device, stream) device scratch (qpb_workspace.hip): `launch`
// receives the buffer (>= bytes) and queues its work on `stream` while the
// cache is locked, so no other thread can grow (free) it in between.
hipError_t qpb_with_workspace(hipStream_t stream, size_t bytes, const std::function<hipError_t(void *)> &launch)
    __attribute__((visibility("hidden")));

namespace qpb {

constexpr double kInf = __builtin_huge_val();

// compile-time unrolled loop: f(std::integral_constant<int, I>) for I = 0..N-1
template <class F, int... I>
__device__ __forceinline__ void unroll_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F &&f) {
  unroll_impl(f, std::make_integer_sequence<int, N>{});
}

// DPP controls (gfx9 encoding)
constexpr int kRowRor = 0x120;       // row_ror:N = 0x120 + N
constexpr int kRowNewBcast = 0x150;  // row_newbcast:J = 0x150 + J (gfx90a+)

// lane J of this 16-lane row, broadcast to the whole row
template <int J>
__device__ __forceinline__ double bc(double v) {
  return __builtin_amdgcn_mov_dpp(v, kRowNewBcast + J, 0xF, 0xF, true);
}
template <int J>
__device__ __forceinline__ int bci(int v) {
  return __builtin_amdgcn_mov_dpp(v, kRowNewBcast + J, 0xF, 0xF, true);
}
template <int N>
__device__ __forceinline__ double ror(double v) {
  return __builtin_amdgcn_mov_dpp(v, kRowRor + N, 0xF, 0xF, true);
}
template <int N>
__device__ __forceinline__ int rori(int v) {
  return __builtin_amdgcn_mov_dpp(v, kRowRor + N, 0xF, 0xF, true);
}

// (value, index) min over the 16 lanes of the row; ties -> smaller index.
// Exact (no rounding), so every lane ends with the identical pair.
template <int N>
__device__ __forceinline__ void argmin_step(double &v, int &i) {
  const double v2 = ror<N>(v);
  const int i2 = rori<N>(i);
  const bool take = (v2 < v) || (v2 == v && i2 < i);
  v = take ? v2 : v;
  i = take ? i2 : i;
}
__device__ __forceinline__ void row_argmin(double &v, int &i) {
  argmin_step<8>(v, i);
  argmin_step<4>(v, i);
  argmin_step<2>(v, i);
  argmin_step<1>(v, i);
}

// Ordering point for LDS traffic between lanes of ONE wavefront.  A wave's DS
// instructions execute in issue order, so only the compiler has to be kept
// from moving LDS accesses across this point; no s_barrier is issued (the
// waves of a workgroup run different trip counts and must never meet).
// Materialise v in a VGPR at this point of the program: IR passes sink pure
// arithmetic towards its uses (past sched_barriers), which in the unrolled
// factorisation sweeps keeps whole broadcast rows alive across steps.
__device__ __forceinline__ void pin(double &v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace qpb

namespace qpb {

// 1/x and 1/sqrt(x) from the hardware estimates (v_rcp_f64 / v_rsq_f64) plus
// two Newton steps: full fp64 accuracy (<= 1 ulp), ~6 instructions instead of
// the IEEE division / sqrt expansions.  Callers guarantee x > 0 finite (or
// discard the result).
__device__ __forceinline__ double rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
  y = __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
  return y;
}
__device__ __forceinline__ double rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * __builtin_fma(-0.5 * x * y, y, 1.5);
  y = y * __builtin_fma(-0.5 * x * y, y, 1.5);
  return y;
}

// ... with one Newton step: the hardware estimates are within 5.3e-8
// (2^-24.2) relative on gfx950 (tools/probe/valu_probe.hip, 1M inputs over
// 200 binades), so one step leaves <= ~3e-15 (2^-48); the n <= 16 kernel uses
// these (-3% kernel time at B = 65,536, interleaved A/B)
__device__ __forceinline__ double rcp1(double x) {
  const double y = __builtin_amdgcn_rcp(x);
  return __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
}
__device__ __forceinline__ double rsq1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * __builtin_fma(-0.5 * x * y, y, 1.5);
}

constexpr double kBig = 1.7976931348623157e308;  // DBL_MAX: the "no candidate" key

// min-reduction key: a finite double whose low 5 mantissa bits carry an index
// (value perturbed by <= 31 ulp).  v_min_f64 over the 16 lanes then yields the
// minimum and its index together, 3 instructions per DPP step.
__device__ __forceinline__ double pack_key(double v, int idx) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double, (b & ~31ull) | (unsigned long long)idx);
}
__device__ __forceinline__ int key_index(double k) {
  return (int)(__builtin_bit_cast(unsigned long long, k) & 31ull);
}
// the same with a 6-bit index (one QP per 64-lane wave)
__device__ __forceinline__ double pack_key64(double v, int idx) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  return __builtin_bit_cast(double, (b & ~63ull) | (unsigned long long)idx);
}
__device__ __forceinline__ int key_index64(double k) {
  return (int)(__builtin_bit_cast(unsigned long long, k) & 63ull);
}
__device__ __forceinline__ double row_min(double v) {
  v = __builtin_fmin(v, ror<8>(v));
  v = __builtin_fmin(v, ror<4>(v));
  v = __builtin_fmin(v, ror<2>(v));
  v = __builtin_fmin(v, ror<1>(v));
  return v;
}

// max of a 32-bit key over the 16 lanes of the row: the DPP moves fuse into
// v_max_u32 (row_ror source modifier), one instruction per step
__device__ __forceinline__ uint32_t row_max_u32(uint32_t v) {
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 8, 0xF, 0xF, true));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 4, 0xF, 0xF, true));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 2, 0xF, 0xF, true));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 1, 0xF, 0xF, true));
  return v;
}

// sum over the 16 lanes of the row by an xor butterfly (quad_perm 1032,
// quad_perm 2301, row_half_mirror, row_mirror): at every level the two
// partners add the same two numbers in swapped order, which IEEE addition
// makes bitwise equal, so all lanes end with the identical sum.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ double row_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return v;
}

// acc += src[lane K of this 16-lane row] * mul: v_fmac_f64 with a DPP
// row_newbcast source operand (gfx950's DP ALU DPP), the broadcast fused into
// the FMA instead of a separate v_mov_b64_dpp.  hipcc neither forms this
// instruction nor pads hazards inside inline asm: callers guarantee that no
// VALU instruction wrote `src` in the two instructions before (the VALU-write
// -> DPP-read hazard), e.g. by an ordering point between the producing step
// and this one (fmac_bc), or use fmac_bc_nop, which issues the 2 wait states.
template <int K>
__device__ __forceinline__ void fmac_bc(double &acc, double src, double mul) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(src), "v"(mul), "i"(K));
}
template <int K>
__device__ __forceinline__ void fmac_bc_nop(double &acc, double src, double mul) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(src), "v"(mul), "i"(K));
}

// exact min over the 16 lanes of the row (v_min_f64 on row_ror moves)
__device__ __forceinline__ double row_min_exact(double v) { return row_min(v); }

// The same without the canonicalising v_max_f64 that fmin() adds behind every
// DPP move (4 fp64 instructions per reduction).  Operands are finite or
// +-inf (never NaN) wherever it is used.
__device__ __forceinline__ double fmin_raw(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double row_min_raw(double v) {
  v = fmin_raw(v, ror<8>(v));
  v = fmin_raw(v, ror<4>(v));
  v = fmin_raw(v, ror<2>(v));
  v = fmin_raw(v, ror<1>(v));
  return v;
}

// Two wait states after the VALU instruction that produced `v`, before a run of
// fmac_bc reads it through DPP (hipcc does not pad hazards around inline asm).
// Taking v as an operand pins its producer above the s_nop.
__device__ __forceinline__ void dpp_ready(double v) { asm volatile("s_nop 1" ::"v"(v)); }
// min of a 32-bit value over the 16 lanes of the row (DPP-fused v_min_u32)
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
  v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 8, 0xF, 0xF, true));
  v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 4, 0xF, 0xF, true));
  v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 2, 0xF, 0xF, true));
  v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kRowRor + 1, 0xF, 0xF, true));
  return v;
}

// max of a per-row-uniform int over the 4 rows of the wave, as a wave-uniform
// (SGPR) value: bounds for skipping dead steps of unrolled loops.
__device__ __forceinline__ int wave_max4(int v) {
  const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  const int ab = a > b ? a : b, cd = c > d ? c : d;
  return ab > cd ? ab : cd;
}
__device__ __forceinline__ int wave_min4(int v) {
  const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  const int ab = a < b ? a : b, cd = c < d ? c : d;
  return ab < cd ? ab : cd;
}

// Diagnostic builds only (STAMP = true, qpb_solve_sections): s_memrealtime stamps
// (100 MHz) accumulate each wave's ticks per kernel section; the real kernels have none.
// A wave adds its counters into the row (blockIdx.x mod kSectionSlots) of a
// kSectionSlots x kSections buffer: one shared row made the flush atomics of a
// 262,144-wave launch serialise on 20 addresses (a 30x longer stamped kernel).
constexpr int kSections = 20;
constexpr int kSectionSlots = 256;
template <bool ON>
struct SectionClock {
  __device__ __forceinline__ void tick(int) {}
  __device__ __forceinline__ void flush(unsigned long long *) {}
};
template <>
struct SectionClock<true> {
  unsigned long long last, acc[kSections];
  __device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  }
  __device__ __forceinline__ SectionClock() {
    for (int i = 0; i < kSections; ++i) acc[i] = 0;
    last = now();
  }
  __device__ __forceinline__ void tick(int i) {
    const unsigned long long t = now();
    acc[i] += t - last;
    last = t;
  }
  __device__ __forceinline__ void flush(unsigned long long *dbg) {
    if ((threadIdx.x & 63) == 0) {
      unsigned long long *row = dbg + (size_t)(blockIdx.x % kSectionSlots) * kSections;
      for (int i = 0; i < kSections; ++i) atomicAdd(&row[i], acc[i]);
    }
  }
};

}  // namespace qpb
