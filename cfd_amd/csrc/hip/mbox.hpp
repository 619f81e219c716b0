// mbox.hpp -- descriptor of the device mailbox used by the one-shot Z-slab
// all-reduce (kernels.hpp mbox_allreduce; set up in slab_comm.hip).
#pragma once

namespace cfdhip {

constexpr int MBOX_MAX = 16;
struct Mbox {
    unsigned long long* slot[MBOX_MAX];  // every rank's mailbox (own one at [rank])
    int n, rank;
    unsigned long long count;            // reductions done (device-side sequence)
    long long timeout_ticks;
};

}  // namespace cfdhip
