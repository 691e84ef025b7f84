// nk_stencil_inst.hip -- instantiates the stencil kernels of ONE problem kind (NK_ST_KIND, set by
// the Makefile: one object per kind, compiled in parallel).
#include "nk_stencil_kern.hpp"

#ifndef NK_ST_KIND
#error "compile with -DNK_ST_KIND=<problem kind>"
#endif
#define NK_CAT2(a, b) a##b
#define NK_CAT(a, b) NK_CAT2(a, b)

namespace nk {

StInst NK_CAT(stencil_kind_, NK_ST_KIND)(const KArgs& A, int mode, int epi, int vec, int grid, hipStream_t s, bool per) {
    return go_stencil_mode<NK_ST_KIND>(A, mode, epi, vec, grid, s, per);
}

hipError_t NK_CAT(stencil_bind_mb_, NK_ST_KIND)(const MbInfo& m) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_mb), &m, sizeof(m));
}

}  // namespace nk
