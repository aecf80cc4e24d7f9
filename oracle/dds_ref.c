/*
 * oracle/dds_ref.c -- TEST INFRASTRUCTURE (oracle_dds) and DDS CPU baseline.
 *
 * Scalar restatement of the build-defined fixed-point DDS.
 * The reference contains no signal generator (it is in the external QubiC
 * gateware, README.md:3); what it does pin is the interface: pulse_iface
 * fields (hdl/pulse_iface.sv:2-6), env buffer words I16|Q16 addressed in
 * 4-sample units (asmparse.py:40-41,46-63; assembler.py:472-476) and freq
 * buffer entries [f/f_clk * 2^32, 15 sub-sample rotations I16|Q16]
 * (asmparse.py:64-86).  Sample parity is therefore pinned only by this file.
 *
 * Channel = (lane, element).  Output sample j of a channel is at cycle
 * n = j / spc, sub-sample k = j % spc:
 *   pulse   latest strobe of the element with t <= n (ties: later event)
 *   env     e = (j - t*spc) / interp; word A*4 + e of the env table
 *           (A = env_word[11:0], L = env_word[23:12] 4-sample words,
 *            e >= 4L ends the pulse; L == 0 is CW: e = 0)
 *   phase   theta = F0 * (n - t_ref) + phase17 << 15  (mod 2^32),
 *           t_ref = latest pulse_reset with t <= n (else 0)
 *   carrier c0 = (cos, sin)(theta) from the Q15 table at theta >> 20
 *           (entries in [-32767, 32767])
 *   amp     a0 = (c0 * amp + 2^15) >> 16           (stays in [-32767, 32767])
 *   rotate  k > 0: a = symsat((a0 (x) R_k + 2^14) >> 15), R_k = freq word k,
 *           symsat = clamp to [-32767, 32767];  k == 0: a = a0
 *   out     sat16((env (x) a + 2^14) >> 15), I and Q
 * (x) = complex product of I16|Q16 words; >> is arithmetic (floor).  Every
 * intermediate fits in int32 (the GPU evaluates each (x) with two
 * v_dot2_i32_i16); this restatement uses int64 and explicit formulas.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

void oracle_dds_sin_lut(int16_t *out)
{
    for (int i = 0; i <= 1024; i++) {
        const int16_t q = (int16_t)lround(32767.0 * sin(2.0 * M_PI * (double)i / 4096.0));
        out[i & 4095] = q;
        if (i < 1024) out[2048 - i] = q;
        out[(2048 + i) & 4095] = (int16_t)-q;
        if (i > 0 && i < 1024) out[4096 - i] = (int16_t)-q;
    }
}

static int32_t clamp(int64_t v, int32_t lo, int32_t hi) { return v > hi ? hi : (v < lo ? lo : (int32_t)v); }

static int64_t asr(int64_t v, int s) { return v >= 0 ? (v >> s) : -((-v + (1ll << s) - 1) >> s); }

/* (a (x) b + 2^14) >> 15, each component clamped to [lo, 32767] */
static void cmul_q15(int32_t ai, int32_t aq, int32_t bi, int32_t bq, int32_t lo, int32_t *oi, int32_t *oq)
{
    *oi = clamp(asr((int64_t)ai * bi - (int64_t)aq * bq + (1 << 14), 15), lo, 32767);
    *oq = clamp(asr((int64_t)ai * bq + (int64_t)aq * bi + (1 << 14), 15), lo, 32767);
}

void oracle_dds(const oracle_dds_args *a, int n_threads)
{
    int16_t lut[4096];
    oracle_dds_sin_lut(lut);
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    #pragma omp parallel for schedule(dynamic, 1)
    for (int64_t ch = 0; ch < (int64_t)a->n_channels; ch++) {
        const uint32_t *d = a->ch + 8 * ch;
        const uint32_t lane = d[0], elem = d[1], spc = d[2], interp = d[3] ? d[3] : 1;
        const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
        uint32_t n_ev = a->summary[8ull * lane + 2];
        if (n_ev > a->event_cap) n_ev = a->event_cap;
        uint32_t *out = a->iq + (uint64_t)ch * a->n_samples;
        /* the latest strobe of the element and the latest pulse_reset at or
         * before cycle n: a lane's events are in time order, so one cursor
         * walks them as n grows (ties: the later event wins) */
        uint32_t e = 0;
        int have = 0;
        uint32_t st_t = 0, env_w = 0, pf = 0, amp = 0, t_ref = 0;
        for (uint32_t j = 0; j < a->n_samples; j++) {
            const uint32_t n = j / spc, k = j % spc;
            for (; e < n_ev; e++) {
                const uint32_t *ev = a->events + 4 * ((uint64_t)e * a->n_lanes + lane);
                if (ev[0] > n) break;
                const uint32_t kind = ev[1] >> 28, cfg = (ev[1] >> 24) & 0xF;
                if (kind == DPEMU_EV_PULSE_RESET) t_ref = ev[0];
                if (kind == DPEMU_EV_STROBE && (cfg & 3) == elem) {
                    have = 1; st_t = ev[0]; env_w = ev[1] & 0xFFFFFF; pf = ev[2]; amp = ev[3] & 0xFFFF;
                }
            }
            int32_t oi = 0, oq = 0;
            if (have) {
                const uint32_t A = env_w & 0xFFF, L = (env_w >> 12) & 0xFFF;
                const uint32_t r = j - st_t * spc;
                const uint32_t es = L ? r / interp : 0;
                const uint32_t widx = 4 * A + es;
                const uint32_t fi = pf >> 17, phase = pf & 0x1FFFF;
                if ((!L || es < 4 * L) && widx < env_len && 16 * fi + 15 < freq_len) {
                    const uint32_t ew = a->env[env_off + widx];
                    const int32_t ei = (int16_t)(ew >> 16), eq = (int16_t)(ew & 0xFFFF);
                    const uint32_t *fr = a->freq + freq_off + 16 * fi;
                    const uint32_t theta = fr[0] * (n - t_ref) + (phase << 15);
                    const uint32_t idx = theta >> 20;
                    const int32_t ci = lut[(idx + 1024) & 4095], cq = lut[idx];
                    int32_t ai = (int32_t)asr((int64_t)ci * amp + (1 << 15), 16);
                    int32_t aq = (int32_t)asr((int64_t)cq * amp + (1 << 15), 16);
                    if (k) {
                        const int32_t ri = (int16_t)(fr[k] >> 16), rq = (int16_t)(fr[k] & 0xFFFF);
                        cmul_q15(ai, aq, ri, rq, -32767, &ai, &aq);
                    }
                    cmul_q15(ei, eq, ai, aq, -32768, &oi, &oq);
                }
            }
            out[j] = (uint32_t)(uint16_t)oi | ((uint32_t)(uint16_t)oq << 16);
        }
    }
}
