// Operand descriptor shared by the MFMA tile engines (gemm_lds.hpp, gemm_sk.hpp).
#pragma once
#include "common.hpp"

namespace dqnx {

enum { L_ROWS_K = 0, L_K_ROWS = 1 };

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
