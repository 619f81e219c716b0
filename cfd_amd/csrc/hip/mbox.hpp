// mbox.hpp -- descriptor of the device mailbox used by the one-shot Z-slab
// all-reduce (kernels.hpp mbox_allreduce; set up in slab_comm.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace cfdhip {

constexpr int MBOX_MAX = 16;
struct Mbox {
    unsigned long long* slot[MBOX_MAX];  // every rank's mailbox (own one at [rank])
    int n, rank;
    unsigned long long count;            // reductions done (device-side sequence)
    long long timeout_ticks;
};

// ---------------------------------------------------------------------------
// One-shot device all-reduce over peer memory (Z-slabs, opt-in): the last
// workgroup of a sweep writes its total into slot [parity][rank] of every
// rank's mailbox (system-scope stores over xGMI), then waits until all ranks'
// slots carry the same sequence number and sums them in rank order, so every
// rank holds the same bits. The sequence counter lives on the device and
// advances only when a reduction actually runs, so consecutive reductions
// alternate parity and a slot is never overwritten before its reader has
// consumed it. take_max: the maximum instead of the sum (L-inf residuals).
// A bounded wait (timeout_ticks of wall_clock64) turns a lost
// peer into a reported error instead of a hung GPU.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool mbox_allreduce(Mbox* mb, double v, double* out,
                                               bool take_max = false) {
    const unsigned long long seq = mb->count + 1;
    mb->count = seq;
    const int n = mb->n, me = mb->rank;
    const int par = (int)(seq & 1ull);
    const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
    for (int r = 0; r < n; ++r) {
        unsigned long long* s = mb->slot[r] + 2 * (par * MBOX_MAX + me);
        __hip_atomic_store(s, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(s + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    unsigned long long* mine = mb->slot[me];
    const long long t0 = wall_clock64();
    double sum = 0.0;
    for (int r = 0; r < n; ++r) {
        unsigned long long* s = mine + 2 * (par * MBOX_MAX + r);
        while (__hip_atomic_load(s + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > mb->timeout_ticks) return false;
        }
        const double x = __longlong_as_double(
            (long long)__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        sum = take_max ? (r == 0 ? x : fmax(sum, x)) : sum + x;
    }
    *out = sum;
    return true;
}

// Two values in one exchange (the single-reduction CG's gamma and delta):
// slots [v0, v1, seq] in a second region of the mailbox, same sequence
// counter (so this and mbox_allreduce alternate parity consistently).
constexpr int MBOX2_BASE = 128;  // u64 offset; the one-value region ends at 64
__device__ __forceinline__ bool mbox_allreduce2(Mbox* mb, double v0, double v1, double* out0,
                                                double* out1) {
    const unsigned long long seq = mb->count + 1;
    mb->count = seq;
    const int n = mb->n, me = mb->rank;
    const int par = (int)(seq & 1ull);
    const unsigned long long b0 = (unsigned long long)__double_as_longlong(v0);
    const unsigned long long b1 = (unsigned long long)__double_as_longlong(v1);
    for (int r = 0; r < n; ++r) {
        unsigned long long* s = mb->slot[r] + MBOX2_BASE + 3 * (par * MBOX_MAX + me);
        __hip_atomic_store(s, b0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(s + 1, b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(s + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    unsigned long long* mine = mb->slot[me];
    const long long t0 = wall_clock64();
    double a0 = 0.0, a1 = 0.0;
    for (int r = 0; r < n; ++r) {
        unsigned long long* s = mine + MBOX2_BASE + 3 * (par * MBOX_MAX + r);
        while (__hip_atomic_load(s + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > mb->timeout_ticks) return false;
        }
        a0 += __longlong_as_double(
            (long long)__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        a1 += __longlong_as_double(
            (long long)__hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
    *out0 = a0;
    *out1 = a1;
    return true;
}

}  // namespace cfdhip
