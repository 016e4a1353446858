// Compact-only instantiations of the persistent greedy kernel for mid-size blocks: 512 threads with FOUR
// or SIX register rows per thread and the rest of the block in LDS (1 280 .. 4 095 rows per block on a
// single launch: config 4's run starts, the LV call's 5e5 rows), plain, batch and guarded.  The
// compact-only kernel carries no exact / mixed sweep, so it runs leaner than the general kernel of the
// same rows (profiles/r05_mid_rows_probe.log).  A translation unit of their own, compiled in parallel
// with persistent.hip.
#include "persistent_kernel.hpp"

namespace st {

namespace {

template <int D, bool GF, int RT>
const void* pick(bool batch, bool guard) {
    if (guard) {
        if (batch) return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 512, 1, true, false, BatchArgs, true>);
        return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 512, 1, true, false, PersistArgs, true>);
    }
    if (batch) return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 512, 1, true, false, BatchArgs>);
    return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 512, 1, true, false>);
}

template <int D, bool GF>
const void* pick_rt(int rt, bool batch, bool guard) {
    if (rt == 4) return pick<D, GF, 4>(batch, guard);
    if (rt == 6) return pick<D, GF, 6>(batch, guard);
    return nullptr;
}

}  // namespace

// the compact-only kernel for a mid-size plan (persistent.hip launch_p, 512 threads, RT 4 / 6), or nullptr
const void* cmp_persistent_fn(int d, bool gf, int rt, bool batch, bool guard) {
    if (d == 2) return gf ? pick_rt<2, true>(rt, batch, guard) : pick_rt<2, false>(rt, batch, guard);
    if (d == 4) return gf ? pick_rt<4, true>(rt, batch, guard) : pick_rt<4, false>(rt, batch, guard);
    return nullptr;
}

}  // namespace st
