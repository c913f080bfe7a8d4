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

#include <utility>

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
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace qpb
