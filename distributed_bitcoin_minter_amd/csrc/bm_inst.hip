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
// BM_INST_PADK_LO..HI (round 6): this unit instantiates ONLY the folded
// padding-block kernels search_kernel_padk<P, K> for K in [LO, HI] and P in
// [BM_INST_PLO, BM_INST_PHI] (messages of 3 to 15 prefix blocks; the Makefile's
// instk_* units), so each of the many such kernels builds in parallel with
// the others.

extern "C" void bm_register_search_kernel(int p, int nbv, const void* fn);

#include <utility>

namespace {
// table slot nbv = 3 + K: the padding-block layouts with their constants
// folded, after K whole prefix blocks (K = 0: search_kernel_padc<P>, a
// one-block message; K = 1, 2: search_kernel_padk<P, K> in the NBV = 1 units,
// K = 3..15 in the instk_* units); NBV = 1 ranges only
#ifdef BM_INST_PADK_LO
template <int P, int K>
void register_padk() {
    static_assert(P >= 55 && K >= BM_INST_PADK_LO && K <= BM_INST_PADK_HI, "padk unit");
    bm_register_search_kernel(P, 3 + K, reinterpret_cast<const void*>(&bm::search_kernel_padk<P, K>));
}
template <int P, int... J>
void register_padk_all(std::integer_sequence<int, J...>) {
    (register_padk<P, BM_INST_PADK_LO + J>(), ...);
}
template <int P>
void register_one() {
    register_padk_all<P>(std::make_integer_sequence<int, BM_INST_PADK_HI - BM_INST_PADK_LO + 1>{});
}
#else
template <int P>
void register_one() {
    bm_register_search_kernel(P, BM_INST_NBV, reinterpret_cast<const void*>(&bm::search_kernel<P, BM_INST_NBV>));
    if constexpr (BM_INST_NBV == 1 && P >= 55) {
        bm_register_search_kernel(P, 3, reinterpret_cast<const void*>(&bm::search_kernel_padc<P>));
        bm_register_search_kernel(P, 4, reinterpret_cast<const void*>(&bm::search_kernel_padk<P, 1>));
        bm_register_search_kernel(P, 5, reinterpret_cast<const void*>(&bm::search_kernel_padk<P, 2>));
    }
}
#endif
template <int... I>
void register_all(std::integer_sequence<int, I...>) {
    (register_one<BM_INST_PLO + I>(), ...);
}
struct Registrar {
    Registrar() { register_all(std::make_integer_sequence<int, BM_INST_PHI - BM_INST_PLO + 1>{}); }
};
const Registrar registrar;
}  // namespace
