// Near-tie guarded instantiations of the persistent greedy kernel (GUARD = true; persistent_kernel.hpp,
// the guard's description above tie_check).  A translation unit of their own, so that they compile in
// parallel with persistent.hip's unguarded kernels -- which carry none of the guard's code.
#include "persistent_kernel.hpp"

namespace st {

namespace {

template <int D, bool GF, int RT, int NT, int BPC, bool GEN>
const void* kernel(bool batch) {
    if (batch) {
        if constexpr (BPC == 1)
            return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, true, GEN, BatchArgs, true>);
        else
            return nullptr;
    }
    return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, true, GEN, PersistArgs, true>);
}

// the plans launch_p instantiates (persistent.hip launch_p_cmp / launch_p_rt), compact arithmetic
template <int D, bool GF>
const void* pick(int rt, int nt, int bpc, bool gen, bool batch) {
    if (!gen) {   // compact-only kernels: 512 threads, 8 register rows (guarded plans use no more: persistent.hip)
        if (nt != 512 || bpc != 1 || rt != 8) return nullptr;
        return kernel<D, GF, 8, 512, 1, false>(batch);
    }
    if (bpc == 2) {
        if (rt <= 4) return kernel<D, GF, 4, 256, 2, true>(batch);
        return kernel<D, GF, 8, 256, 2, true>(batch);
    }
    if (nt == 512) {
        if (rt <= 4) return kernel<D, GF, 4, 512, 1, true>(batch);
        if (rt <= 6) return kernel<D, GF, 6, 512, 1, true>(batch);
        return kernel<D, GF, 8, 512, 1, true>(batch);
    }
    switch (rt) {
        case 4: return kernel<D, GF, 4, 256, 1, true>(batch);
        case 8: return kernel<D, GF, 8, 256, 1, true>(batch);
        default: return kernel<D, GF, 16, 256, 1, true>(batch);
    }
}

}  // namespace

const void* guarded_persistent_fn(int d, bool gf, int rt, int nt, int bpc, bool gen, bool batch) {
    if (d == 2) return gf ? pick<2, true>(rt, nt, bpc, gen, batch) : pick<2, false>(rt, nt, bpc, gen, batch);
    if (d == 4) return gf ? pick<4, true>(rt, nt, bpc, gen, batch) : pick<4, false>(rt, nt, bpc, gen, batch);
    return nullptr;
}

}  // namespace st
