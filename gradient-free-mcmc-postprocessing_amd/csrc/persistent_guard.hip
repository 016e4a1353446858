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
    if (bpc != 1) return nullptr;
    if (!gen) {   // compact-only kernels: 512 threads, 8 register rows (9 only when st_tune key 12 asks: persistent.hip)
        if (nt != 512) return nullptr;
        // 4 register rows: the guarded mid-size plan (1 280 .. 4 095 rows per block, one thin at a time) --
        // the general kernel of 4 rows spills under the guard (28 B of scratch at d = 4), this one does not
        if (rt == 4) return batch ? nullptr : kernel<D, GF, 4, 512, 1, false>(false);
        if (rt < 8 || rt > 9) return nullptr;
        return rt == 9 ? kernel<D, GF, 9, 512, 1, false>(batch) : kernel<D, GF, 8, 512, 1, false>(batch);
    }
    if (nt == 512) {
        if (rt <= 4) return kernel<D, GF, 4, 512, 1, true>(batch);
        return kernel<D, GF, 8, 512, 1, true>(batch);
    }
    return rt == 4 ? kernel<D, GF, 4, 256, 1, true>(batch) : nullptr;   // (1 / 2 rows: persistent_small.hip)
}

}  // namespace

const void* guarded_persistent_fn(int d, bool gf, int rt, int nt, int bpc, bool gen, bool batch) {
    if (d == 2) return gf ? pick<2, true>(rt, nt, bpc, gen, batch) : pick<2, false>(rt, nt, bpc, gen, batch);
    if (d == 4) return gf ? pick<4, true>(rt, nt, bpc, gen, batch) : pick<4, false>(rt, nt, bpc, gen, batch);
    return nullptr;
}

}  // namespace st
