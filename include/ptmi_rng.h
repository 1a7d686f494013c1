/*
 * ptmi_rng.h — the counter-based random stream shared by the HIP kernels and
 * the CPU oracle.
 *
 * The reference draws with ti.random() (kernels.py:21, 33, 47-48, 184-185,
 * 441, 894, 1150, 1388): a per-thread stateful generator whose stream depends
 * on the backend and on thread scheduling and has no seed in the repo
 * (SURVEY.md §8c), so it cannot be reproduced. This header replaces it with a
 * stream that is a pure function of (seed, pixel, sample, draw#):
 *
 *   key      = pt_path_key(seed, pixel, sample)     once per camera path
 *   u_n      = pt_rand(key, n), n = 0, 1, 2, ...    the n-th ti.random()
 *
 * Draw numbers advance in exactly the order the reference calls ti.random()
 * along one path, so a path's random numbers do not depend on which thread,
 * wave, queue slot or GPU processes it: megakernel, wavefront, tile-sharded
 * and CPU-oracle runs of the same path consume the same values.
 * Outputs are multiples of 2^-24 in [0, 1), exact in f32.
 */
#ifndef PTMI_RNG_H
#define PTMI_RNG_H

#include <stdint.h>
#include "ptmi_math.h"

/* 32-bit finalizer (2 multiply / 3 xor-shift rounds, "lowbias32"). */
PT_HD uint32_t pt_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

PT_HD uint32_t pt_path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t h = pt_mix32(seed + 0x68e31da4u);
    h = pt_mix32(h ^ (pixel * 0x9e3779b9u));
    h = pt_mix32(h + (sample * 0x85ebca6bu) + 0xc2b2ae35u);
    return h;
}

PT_HD uint32_t pt_rand_u32(uint32_t key, uint32_t n) {
    return pt_mix32(key ^ pt_mix32(n * 0x9e3779b9u + 0x632be5abu));
}

PT_HD float pt_rand(uint32_t key, uint32_t n) {
    return (float)(pt_rand_u32(key, n) >> 8) * 5.9604644775390625e-8f; /* 2^-24 */
}

#endif /* PTMI_RNG_H */
