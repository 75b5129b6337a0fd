// bm_inst.hip -- explicit instantiations of search_kernel<P, NBV> for
// P in [BM_INST_PLO, BM_INST_PHI] and NBV = BM_INST_NBV (and of
// search_kernel_padc<P> / search_kernel_padk<P, K> for the padding-block
// P >= 55), registered into the
// launcher's table at load time.  The Makefile compiles this file once per
// P range (in parallel) so a full build of all 83 layouts stays short.
#include "bm_kernels.hpp"

#if !defined(BM_INST_PLO) || !defined(BM_INST_PHI) || !defined(BM_INST_NBV)
#error "define BM_INST_PLO, BM_INST_PHI and BM_INST_NBV"
#endif

extern "C" void bm_register_search_kernel(int p, int nbv, const void* fn);

#include <utility>

namespace {
// table slot nbv = 3 + K: the padding-block layouts with their constants
// folded, after K whole prefix blocks (K = 0: search_kernel_padc<P>, a
// one-block message; K = 1, 2: search_kernel_padk<P, K>); NBV = 1 ranges only
template <int P>
void register_one() {
    bm_register_search_kernel(P, BM_INST_NBV, reinterpret_cast<const void*>(&bm::search_kernel<P, BM_INST_NBV>));
    if constexpr (BM_INST_NBV == 1 && P >= 55) {
        bm_register_search_kernel(P, 3, reinterpret_cast<const void*>(&bm::search_kernel_padc<P>));
        bm_register_search_kernel(P, 4, reinterpret_cast<const void*>(&bm::search_kernel_padk<P, 1>));
        bm_register_search_kernel(P, 5, reinterpret_cast<const void*>(&bm::search_kernel_padk<P, 2>));
    }
}
template <int... I>
void register_all(std::integer_sequence<int, I...>) {
    (register_one<BM_INST_PLO + I>(), ...);
}
struct Registrar {
    Registrar() { register_all(std::make_integer_sequence<int, BM_INST_PHI - BM_INST_PLO + 1>{}); }
};
const Registrar registrar;
}  // namespace
