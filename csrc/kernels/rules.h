// Device interpreter of the routing rule program (ccfd_abi.h ccfd_rule_prog, compiled by
// router/rules.py RuleSet.device_program): the reference's configurable Drools routing
// rules (README.md:427, deploy/router.yaml:69-70) evaluated per row inside the fused
// scoring kernels, so non-threshold rule sets keep the GPU-side route byte, counters,
// amount histogram and compacted fraud list exact.
//
// The program is wave-uniform (scalar loads, uniform control flow): every lane runs every
// op for its own row, so operand gathers across the lane groups of a row (__shfl) are
// legal.  The stack lives in 8 named registers addressed by the wave-uniform stack pointer
// (select chains, no scratch).  Arithmetic is IEEE f32 with explicit round-to-nearest ops
// (no FMA contraction), matching RuleSet.evaluate's float32 numpy evaluation.
#pragma once
#include "common.h"

namespace ccfd {

struct RuleStack {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, s5 = 0.f, s6 = 0.f, s7 = 0.f;
  int sp = 0;    // wave-uniform

  __device__ __forceinline__ void push(float v) {
    s0 = sp == 0 ? v : s0; s1 = sp == 1 ? v : s1; s2 = sp == 2 ? v : s2; s3 = sp == 3 ? v : s3;
    s4 = sp == 4 ? v : s4; s5 = sp == 5 ? v : s5; s6 = sp == 6 ? v : s6; s7 = sp == 7 ? v : s7;
    ++sp;
  }
  __device__ __forceinline__ float pop() {
    --sp;
    return sp == 0 ? s0 : sp == 1 ? s1 : sp == 2 ? s2 : sp == 3 ? s3 :
           sp == 4 ? s4 : sp == 5 ? s5 : sp == 6 ? s6 : s7;
  }
};

// `feat(j)` returns canonical feature j (0 = Time, 1..28 = V1..V28, 29 = Amount) of this
// lane's row; it is called with a wave-uniform j from uniform control flow.
template <class Feat>
__device__ __forceinline__ bool rule_route(const ccfd_rule_prog* __restrict__ prog, float p, Feat&& feat) {
  const int nops = prog->n_ops;
  RuleStack st;
  bool decided = false, fraud = prog->default_route != 0;
  for (int i = 0; i < nops; ++i) {
    const ccfd_rule_op op = prog->ops[i];
    const int code = op.op;
    if (code == CCFD_RULE_VAR) {
      st.push(op.arg == 0 ? p : feat(op.arg - 1));
    } else if (code == CCFD_RULE_CONST) {
      st.push(op.imm);
    } else if (code == CCFD_RULE_END) {
      const bool cond = st.pop() != 0.f;
      fraud = (!decided && cond) ? (op.arg != 0) : fraud;
      decided = decided || cond;
    } else if (code == CCFD_RULE_NEG || code == CCFD_RULE_ABS || code == CCFD_RULE_LOG1P || code == CCFD_RULE_NOT) {
      const float a = st.pop();
      float r;
      if (code == CCFD_RULE_NEG) r = -a;
      else if (code == CCFD_RULE_ABS) r = fabsf(a);
      else if (code == CCFD_RULE_LOG1P) r = log1pf(a);
      else r = a == 0.f ? 1.f : 0.f;
      st.push(r);
    } else {
      const float b = st.pop();
      const float a = st.pop();
      float r;
      switch (code) {
        case CCFD_RULE_ADD: r = __fadd_rn(a, b); break;
        case CCFD_RULE_SUB: r = __fsub_rn(a, b); break;
        case CCFD_RULE_MUL: r = __fmul_rn(a, b); break;
        case CCFD_RULE_DIV: r = __fdiv_rn(a, b); break;
        case CCFD_RULE_MIN: r = fminf(a, b); break;
        case CCFD_RULE_MAX: r = fmaxf(a, b); break;
        case CCFD_RULE_GT: r = a > b ? 1.f : 0.f; break;
        case CCFD_RULE_GE: r = a >= b ? 1.f : 0.f; break;
        case CCFD_RULE_LT: r = a < b ? 1.f : 0.f; break;
        case CCFD_RULE_LE: r = a <= b ? 1.f : 0.f; break;
        case CCFD_RULE_EQ: r = a == b ? 1.f : 0.f; break;
        case CCFD_RULE_NE: r = a != b ? 1.f : 0.f; break;
        case CCFD_RULE_AND: r = (a != 0.f && b != 0.f) ? 1.f : 0.f; break;
        case CCFD_RULE_OR: r = (a != 0.f || b != 0.f) ? 1.f : 0.f; break;
        default: r = 0.f; break;
      }
      st.push(r);
    }
  }
  return fraud;
}

__device__ __forceinline__ float sel8(const float xv[8], int s) {
  return s == 0 ? xv[0] : s == 1 ? xv[1] : s == 2 ? xv[2] : s == 3 ? xv[3] :
         s == 4 ? xv[4] : s == 5 ? xv[5] : s == 6 ? xv[6] : xv[7];
}

// Feature j of row c when the four 16-lane groups hold 8 features each:
//   f32 rows (reference column order): group j / 8, slot j % 8;
//   W64 rows (wire order V1..V28, Time, Amount): V_k -> (k-1) / 8, (k-1) % 8; Time -> (3, 4);
//   Amount -> (3, 5).
template <bool kWire>
__device__ __forceinline__ float lane_feature(const float xv[8], int j, int c) {
  int gj, sj;
  if constexpr (kWire) {
    if (j == 0) { gj = 3; sj = 4; }
    else if (j == 29) { gj = 3; sj = 5; }
    else { gj = (j - 1) >> 3; sj = (j - 1) & 7; }
  } else {
    gj = j >> 3; sj = j & 7;
  }
  return __shfl(sel8(xv, sj), gj * 16 + c);
}

}  // namespace ccfd
