// Operand descriptor shared by the MFMA tile engines (gemm_lds.hpp, gemm_sk.hpp).
#pragma once
#include "common.hpp"

namespace dqnx {

// L_ROWS_KU / L_ROWS_K2 (L_K_ROWSU / L_K_ROWS2): the ROWS_K (K_ROWS) image loaded with
// unconditional loads (an element outside the operand reads a valid address and is zeroed by a
// select, so the compiler's vmcnt waits stay exact and no load sits under a branch), as float4
// (the VEC layouts' conditions) or as float2 pairs (ld and K / the column count even: rows
// 8-byte aligned, e.g. the HEAD net's 1358-wide dense-1 weight rows); ROWS_K*: no copy, no gather
enum { L_ROWS_K = 0, L_K_ROWS = 1, L_ROWS_KU = 2, L_ROWS_K2 = 3, L_K_ROWSU = 4, L_K_ROWS2 = 5 };

// One GEMM operand in global memory.
//   ROWS_K: element (r, k) = base[rowidx(r)*ld + k], rowidx(r) = gather ? gather[r] : r;
//           rows r < nrows, k < K (K multiple of 4 when VEC).  copy != null: the loaded
//           fragments are also written to copy[r*ldcopy + k] (layer-1 x materialisation).
//   K_ROWS: element (k, c) = base[k*ld + c], k < K, c < nrows; column `aug` reads 1.0
//           (ones column: a bias gradient is one more GEMM column).
struct Operand {
    const float* base;
    int ld;
    const int32_t* gather;
    int nrows;
    int K;
    int aug;
    float* copy;
    int ldcopy;
};

}  // namespace dqnx
