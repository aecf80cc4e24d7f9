/*
 * oracle/readout.c -- TEST INFRASTRUCTURE.  Scalar restatement of the
 * build-defined readout demodulation model (meas_model DPEMU_MEAS_DEMOD,
 * include/dpemu.h dpemu_config), SURVEY.md §8(f)2: "rdlo demod
 * -> discriminator -> meas/meas_valid".  The reference has no readout model
 * (the cocotb testbenches drive meas / meas_valid by hand,
 * cocotb/fproc_meas/test_meas.py:19-83), so parity is pinned by this file
 * alone; what the reference does fix is the interface: the rdrv / rdlo
 * elements of a qubit (python/test/channel_config.json:13,28-38; rdlo at 4
 * samples per clock into accbuf, hwconfig.py:128,138-140), the DDS phase
 * words (phase17, the freq buffer's f / f_clk * 2^32, asmparse.py:64-86) and
 * the measurement hold (hwconfig.py:9, FPROC_MEAS_CLKS; ir/passes.py:539-548).
 *
 * Integer arithmetic only (both this file and csrc/lane.h demod_readout):
 *
 *   sin33(x)  = sin(2 pi x / 2^33) * 2^61, int64, from a degree-11 odd Taylor
 *               polynomial on the quarter wave in Q30 (relative accuracy ~1e-7
 *               next to every zero, so the Dirichlet ratio below stays exact
 *               to the polynomial's precision for any detuning)
 *   window    n_lo = L_lo * ro_cpw (L = env word bits 23:12; 0 = CW = 4096)
 *   overlap   [a, e) = [t_lo, t_lo + n_lo) n [t_d + delay, t_d + delay + n_d)
 *   phases    beta  = F_d - F_lo                                  (mod 2^32)
 *             alpha = beta (a - t_ref) - F_d delay + (ph_d - ph_lo) << 15
 *                     + theta[s]                                  (mod 2^32)
 *   sum       sum_{k<n} e^{i (alpha + k beta)} = D e^{i gamma}, b = (int32) beta:
 *             gamma = alpha + ((n - 1) b >> 1),  D = sin(n b pi/2^32) / sin(b pi/2^32)
 *             D_q16 = +-((|sin33(n b)| >> sh) << 16) / (|sin33(b)| >> sh), sh
 *             normalising the divisor below 2^31; b = 0: D_q16 = n << 16
 *   signal    M = ((amp_d gain[s]) >> 16) * D_q16
 *             I = (M * c15 + 2^31) >> 32, Q = (M * s15 + 2^31) >> 32, with
 *             c15 / s15 = (sin33(2 gamma + 2^31) / sin33(2 gamma) + 2^45) >> 46
 *             (per clock: amp / 2 in Q15 units, so |acc| < 2^30)
 *   noise     u0..u3 = 16-bit halves of Philox words 1, 2 (word 0 is the state
 *             draw): z_I = u0 + u1 - u2 - u3, z_Q = u0 - u1 + u2 - u3
 *             acc += (z * ro_sigma) >> 16                      (ro_sigma < 2^24)
 *   decide    x = (acc_I axis_I + acc_Q axis_Q) >> 15, outcome = x > ro_thr
 */
#include "oracle.h"

/* sin(pi/2 t) / t = sum_k C_k t^2k, Taylor, Q30 */
static const int64_t SIN_C[6] = {1686629713, -693598668, 85569306, -5026995, 172272, -3864};

int64_t oracle_sin33(int64_t x)
{
    const uint64_t r = (uint64_t)x & ((1ull << 33) - 1);
    const uint32_t q = (uint32_t)(r >> 31);                  /* quadrant */
    const uint64_t f = r & 0x7FFFFFFFull;
    const uint64_t y = (q & 1) ? (1ull << 31) - f : f;       /* Q31 of the quarter wave, <= 2^31 */
    const int64_t z = (int64_t)((y * y) >> 32);              /* t^2, Q30 */
    int64_t p = SIN_C[5];
    for (int k = 4; k >= 0; k--) p = SIN_C[k] + ((p * z) >> 30);
    const int64_t s = (int64_t)y * p;                        /* Q61 */
    return (q & 2) ? -s : s;
}

int64_t oracle_dirichlet_q16(uint32_t n, uint32_t beta)
{
    if (n == 0) return 0;
    const int32_t b = (int32_t)beta;
    if (b == 0) return (int64_t)n << 16;
    const int64_t den = oracle_sin33((int64_t)b);            /* |angle| <= pi/2: no zero but b = 0 */
    const int64_t num = oracle_sin33((int64_t)n * b);
    uint64_t ad = (uint64_t)(den < 0 ? -den : den), an = (uint64_t)(num < 0 ? -num : num);
    int sh = 0;
    while ((ad >> sh) >= (1ull << 31)) sh++;
    ad >>= sh;
    an >>= sh;
    const int64_t q = (int64_t)((an << 16) / ad);
    return ((num < 0) != (den < 0)) ? -q : q;
}

static int64_t q15_of(int64_t s61) { return (s61 + (1ll << 45)) >> 46; }

uint32_t oracle_demod(const dpemu_config *cfg, uint64_t shot, uint32_t core, uint32_t m, uint32_t t_lo,
                      uint32_t env_lo, uint32_t pp_lo, uint32_t f_lo, const oracle_ro_drive *d, uint32_t f_d,
                      uint32_t t_ref, int32_t acc[2])
{
    uint32_t r[4];
    oracle_philox4(cfg->seed, shot, core, m, r);
    const uint32_t thr = cfg->p1_threshold[core];
    const uint32_t s = (thr == 0xFFFFFFFFu) || (r[0] < thr);
    int64_t sig_i = 0, sig_q = 0;
    if (d->have) {
        const uint64_t n_lo = (uint64_t)oracle_ro_words(env_lo) * cfg->ro_cpw;
        const uint64_t n_d = (uint64_t)oracle_ro_words(d->env) * cfg->ro_cpw;
        const uint64_t r0 = (uint64_t)d->t + cfg->ro_delay;  /* the return starts */
        const uint64_t a = r0 > t_lo ? r0 : t_lo;
        const uint64_t e0 = (uint64_t)t_lo + n_lo, e1 = r0 + n_d;
        const uint64_t e = e0 < e1 ? e0 : e1;
        const uint32_t n = e > a ? (uint32_t)(e - a) : 0u;
        if (n) {
            const uint32_t beta = f_d - f_lo;
            const uint32_t alpha = beta * (uint32_t)(a - t_ref) - f_d * cfg->ro_delay +
                                   (((d->pp & 0x1FFFFu) - (pp_lo & 0x1FFFFu)) << 15) + cfg->ro_theta[s];
            const uint32_t gamma = alpha + (uint32_t)(uint64_t)(((int64_t)(n - 1) * (int32_t)beta) >> 1);
            const int64_t dq = oracle_dirichlet_q16(n, beta);
            const int64_t c15 = q15_of(oracle_sin33((int64_t)(((uint64_t)gamma << 1) + (1ull << 31))));
            const int64_t s15 = q15_of(oracle_sin33((int64_t)((uint64_t)gamma << 1)));
            const int64_t amp = (int64_t)(((uint64_t)(d->amp & 0xFFFFu) * cfg->ro_gain[s]) >> 16);
            const int64_t M = amp * dq;
            sig_i = (M * c15 + (1ll << 31)) >> 32;
            sig_q = (M * s15 + (1ll << 31)) >> 32;
        }
    }
    const int32_t u0 = (int32_t)(r[1] & 0xFFFFu), u1 = (int32_t)(r[1] >> 16);
    const int32_t u2 = (int32_t)(r[2] & 0xFFFFu), u3 = (int32_t)(r[2] >> 16);
    const int64_t zi = u0 + u1 - u2 - u3, zq = u0 - u1 + u2 - u3;
    acc[0] = (int32_t)(sig_i + ((zi * (int64_t)cfg->ro_sigma) >> 16));
    acc[1] = (int32_t)(sig_q + ((zq * (int64_t)cfg->ro_sigma) >> 16));
    const uint32_t ax = cfg->ro_axis[core];
    const int64_t x = ((int64_t)acc[0] * (int16_t)(ax & 0xFFFFu) + (int64_t)acc[1] * (int16_t)(ax >> 16)) >> 15;
    return x > (int64_t)cfg->ro_thr;
}

uint32_t oracle_ro_words(uint32_t env)
{
    const uint32_t L = (env >> 12) & 0xFFFu;
    return L ? L : 4096u;
}

uint32_t oracle_ro_freq(const uint32_t *tab, uint32_t len, uint32_t pp)
{
    const uint32_t i = (pp >> 17) & 0x1FFu;
    return (tab && i < len) ? tab[i] : 0u;
}

uint32_t oracle_demod_valid(const dpemu_config *cfg, uint32_t t_lo, uint32_t env_lo, uint32_t last_tv)
{
    const uint32_t tv = t_lo + oracle_ro_words(env_lo) * cfg->ro_cpw + cfg->meas_latency;
    return tv > last_tv ? tv : last_tv + 1u;
}
