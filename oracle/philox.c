/*
 * oracle/philox.c -- TEST INFRASTRUCTURE.  Philox4x32-10 (Salmon et al.,
 * SC'11), the counter-based RNG of the build-defined measurement model:
 * key = seed, counter = (shot_lo, shot_hi, core, measurement index); the
 * outcome draw is output word 0.  Independent of sharding and GPU count.
 */
#include "oracle.h"

static void philox_round(uint32_t ctr[4], const uint32_t key[2])
{
    uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ ctr[1] ^ key[0];
    uint32_t n2 = hi0 ^ ctr[3] ^ key[1];
    ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
}

void oracle_philox4(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m, uint32_t out[4])
{
    uint32_t ctr[4] = {(uint32_t)shot, (uint32_t)(shot >> 32), core, m};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int r = 0; r < 10; r++) {
        philox_round(ctr, key);
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
    for (int i = 0; i < 4; i++) out[i] = ctr[i];
}

uint32_t oracle_philox_u32(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m)
{
    uint32_t r[4];
    oracle_philox4(seed, shot, core, m, r);
    return r[0];
}

/* Measurement outcome (build-defined model, parity unpinned by the reference:
 * the reference testbench drives meas / meas_valid by hand).
 *   state   = thr == 0xFFFFFFFF || r0 < thr          (the prepared qubit state)
 *   STATE   : outcome = state
 *   READOUT : the rdlo demodulation integrated over the window and projected on
 *             the discriminator axis, x = +-(ro_sep * amp >> 16) + (z * ro_sigma >> 16)
 *             with z = Irwin-Hall(4) of the 16-bit halves of r1, r2, centred
 *             (|z| <= 131070, sigma 37837.6); outcome = x > ro_thr.  A weaker
 *             readout pulse (amp word) separates the states less; with ro_win
 *             a window shorter than ro_win env words (env bits 23:12) does too. */
uint32_t oracle_meas_bit(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m, uint32_t thr, uint32_t amp,
                         uint32_t meas_model, int32_t ro_sep, uint32_t ro_sigma, int32_t ro_thr,
                         uint32_t ro_win, uint32_t env)
{
    uint32_t r[4];
    oracle_philox4(seed, shot, core, m, r);
    uint32_t state = (thr == 0xFFFFFFFFu) || (r[0] < thr);
    if (meas_model != DPEMU_MEAS_READOUT) return state;
    int64_t z = (int64_t)(r[1] & 0xFFFFu) + (r[1] >> 16) + (r[2] & 0xFFFFu) + (r[2] >> 16) - 131070;
    int64_t s = ((int64_t)ro_sep * (int64_t)(amp & 0xFFFFu)) >> 16;
    const uint32_t w = (env >> 12) & 0xFFFu;
    if (ro_win && w) {   /* window: (s * min(W, ro_win) * floor(2^24 / ro_win)) >> 24, W = env bits 23:12;
                            W = 0 is a CW envelope (plays until the next pulse): no scaling */
        s = (s * (int64_t)((w < ro_win ? w : ro_win) * ((1u << 24) / ro_win))) >> 24;
    }
    int64_t x = (state ? s : -s) + ((z * (int64_t)ro_sigma) >> 16);
    return x > (int64_t)ro_thr;
}
