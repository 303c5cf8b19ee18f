// mlp_fused.h — fused fp32-MFMA path of the V_hypothesis KFP residual (internal interface).
#pragma once
#include "common.h"

namespace pdeinv {
namespace mlpf {

// Shapes the fused path handles (else the rocBLAS path runs).
bool supported(int d, int L, int W, int O);

// Workspace (floats) for chunks of Bc rows.
size_t workspace_floats(int d, int L, int W, int O, int64_t Bc);

// Per-set loss hook: the orchestrator computes g [R x d] and the per-row terms (V', V''), then
// calls this to accumulate the loss slots and write abar0 = 2 c1 g [R x d] (mlp.hip's loss kernel).
// terms[r] = {V', V'', V, 0}.
struct LossHook {
  int (*fn)(void* ctx, const float* g, const float4* terms, float* abar0, int64_t R, hipStream_t st);
  void* ctx;
};

struct Chunk {
  int d, L, W, O;
  int64_t R;                 // rows in this chunk
  const float* z;            // rows [x | v], stride ldz
  int64_t ldz;
  const float* params;       // flat flax order
  float* grad;               // accumulated (+=)
  const int64_t* poff;       // kernel offsets per layer (0..L)
  const int64_t* boff;       // bias offsets per layer (0..L)
  float c2, c3, c0;          // loss weights of V'', V' and V for this set
  float* ws;                 // workspace_floats(..., Bc >= R)
  int64_t Bc;
  // KMV pair rows (pdeinv_residual_kmv_mlp): per-row value weight w_r = wrow[r * ldw] multiplying c0
  // (nullptr: 1), and grad_only = stop after g = grad_x V of every row (pass 1), left in grad_rows()
  const float* wrow = nullptr;
  int64_t ldw = 0;
  bool grad_only = false;
  // first_order: the set weights only V' (and V) — no |g|^2, no V'', no input-gradient seed (the KFP initial /
  // terminal sets, kinetic_fokker_planck.py:34-39): R1 (g = grad_x V) and F2 (the forward adjoint of abar0 = 0)
  // are skipped, and g, the a planes, a1 and the zetabar planes are zeroed so the later products see exact zeros
  bool first_order = false;
};

// g = grad_x V [R x d] of the last run_chunk (workspace view)
const float* grad_rows(const Chunk& c);

int run_chunk(const Chunk& c, const LossHook& loss, hipStream_t st);

}  // namespace mlpf
}  // namespace pdeinv
