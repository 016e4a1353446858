// Small-shard instantiations of the persistent greedy kernel: 256-thread blocks with ONE or TWO register
// rows per thread, for blocks of at most 256 / 512 rows (config 2's run starts: 47 279 rows on 185 blocks
// of 256; the LV call's run starts: ~118 000 rows, 461 per block).  The default plan's floor of four
// register rows made three of every four rows padding that computes like a real row.  Plain, batch and
// guarded forms; a translation unit of their own, compiled in parallel with persistent.hip.
#include "persistent_kernel.hpp"

namespace st {

namespace {

template <int D, bool GF, int RT>
const void* pick(bool cmp, bool batch, bool guard) {
    if (guard) {
        if (batch) return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 256, 1, true, true, BatchArgs, true>);
        return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 256, 1, true, true, PersistArgs, true>);
    }
    if (batch) {
        if (!cmp) return nullptr;   // batch launches run the compact arithmetic only
        return reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 256, 1, true, true, BatchArgs>);
    }
    return cmp ? reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 256, 1, true>)
               : reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, 256, 1, false>);
}

template <int D, bool GF>
const void* pick_rt(int rt, bool cmp, bool batch, bool guard) {
    if (rt == 1) return pick<D, GF, 1>(cmp, batch, guard);
    if (rt == 2) return pick<D, GF, 2>(cmp, batch, guard);
    return nullptr;
}

}  // namespace

// the kernel for a small-shard plan (persistent.hip launch_p, RT < 4), or nullptr
const void* small_persistent_fn(int d, bool gf, int rt, bool cmp, bool batch, bool guard) {
    if (d == 2) return gf ? pick_rt<2, true>(rt, cmp, batch, guard) : pick_rt<2, false>(rt, cmp, batch, guard);
    if (d == 4) return gf ? pick_rt<4, true>(rt, cmp, batch, guard) : pick_rt<4, false>(rt, cmp, batch, guard);
    return nullptr;
}

}  // namespace st
