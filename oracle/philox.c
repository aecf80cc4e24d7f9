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

uint32_t oracle_philox_u32(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m)
{
    uint32_t ctr[4] = {(uint32_t)shot, (uint32_t)(shot >> 32), core, m};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int r = 0; r < 10; r++) {
        philox_round(ctr, key);
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
    return ctr[0];
}
