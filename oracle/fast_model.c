/*
 * oracle/fast_model.c -- TEST INFRASTRUCTURE (oracle_fast) and CPU baseline.
 *
 * Event-driven restatement of the gateware: each instruction advances its
 * core's next-DECODE cycle by the closed form SURVEY.md §2.4 derives from
 * hdl/ctrl.v (MEM_WAIT/mem_wait_cycles, DECODE, ALU_PROC_0/1, FPROC_WAIT,
 * SYNC_WAIT, QCLK_RST), instead of evaluating every clock:
 *
 *   PULSE_WRITE, PULSE_RESET   D' = D + 3
 *   PULSE_WRITE_TRIG, IDLE     D' = tT + 3, tT = first cycle >= D with
 *                              qclk == cmd_time (strobe visible at tT + 2)
 *   REG_ALU, INC_QCLK, JUMP_I  D' = D + 4 (INC_QCLK: qclk(D+3) = alu + 3)
 *   JUMP_COND                  D' = D + 6
 *   ALU_FPROC / JUMP_FPROC     D' = R + 4 / R + 6, R = fproc ready cycle
 *   SYNC                       D' = S + 3, qclk(S + 2) = 0
 *   DONE / 0000                halt; 1101..1111 hang in DECODE
 *
 * Cores of a shot interact only through measurements (fproc) and the sync
 * barrier; the shot is advanced by always executing the core whose next
 * DECODE is earliest, so every measurement a read can observe is already
 * known.  tests/test_fast_vs_rtl.py pins this file to rtl_model.c.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, as the checker / CPU baseline.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MEAS_LOOKUP DPEMU_MEAS_LOOKUP   /* measurements per core visible to fproc */
#define LUT_FIRE_CAP DPEMU_LUT_FIRE_CAP /* meas_lut fires recorded per shot */
#define INF32 0xFFFFFFFFu

enum { M_RUN = 0, M_SYNC = 1, M_LUT = 2, M_FIN = 3 };

typedef struct {
    const uint32_t *prog; uint32_t n_instr;
    uint32_t ip, t, qa_t, qa_q;
    uint32_t regs[16];
    uint32_t pr[5];                  /* env, phase, freq, amp, cfg */
    int mode; uint32_t wait_d;       /* SYNC / LUT: decode cycle of the waiting instruction */
    uint32_t status, flags, n_instr_exec, n_events, n_trace, n_meas, meas_bits, last_bit;
    uint32_t t_end, ip_end, qclk_end;
    uint32_t mt[MEAS_LOOKUP]; uint8_t mb[MEAS_LOOKUP];   /* measurement (valid cycle, bit) */
    uint32_t lane;                   /* output lane index (cfg->lane_order) */
    uint32_t core;
    /* DEMOD (oracle/readout.c): the latest readout-drive strobe and pulse_reset,
     * the last meas_valid, the program's drive / LO frequency tables */
    oracle_ro_drive ro_d;
    uint32_t ro_tref, ro_last_tv;
    const uint32_t *ro_tab[2]; uint32_t ro_len[2];
} flane;

typedef struct {
    const dpemu_config *cfg;
    const dpemu_outputs *out;
    uint64_t n_lanes;
    uint64_t shot;
    uint32_t C, addr_mask;
    uint64_t part;                   /* sync participants */
    /* meas_lut */
    int lut_ready_next;              /* last fire cycle + 1 is LUT_READY */
    uint32_t lut_last_fire;
    uint64_t lut_valid, lut_addr;
    uint32_t lut_done_until;         /* events with valid <= this applied */
    int lut_any;
    uint32_t lut_cursor[DPEMU_MAX_CORES];
    uint32_t nfire; uint32_t fire_t[LUT_FIRE_CAP]; uint64_t fire_out[LUT_FIRE_CAP];
    flane L[DPEMU_MAX_CORES];
} fshot;

static uint32_t fbits(const uint32_t w[4], int lo, int width)
{
    uint64_t acc = w[lo >> 5];
    if ((lo >> 5) < 3) acc |= (uint64_t)w[(lo >> 5) + 1] << 32;
    acc >>= (lo & 31);
    return (uint32_t)(acc & ((width == 32) ? 0xFFFFFFFFull : ((1ull << width) - 1)));
}

static uint32_t qclk_at(const flane *l, uint32_t t)
{
    return (t < l->qa_t) ? 0u : l->qa_q + (t - l->qa_t);
}

static void emit_event(fshot *s, flane *l, uint32_t t, uint32_t kind)
{
    const dpemu_config *cfg = s->cfg;
    if (l->n_events < cfg->event_cap) {
        if (s->out->events) {     /* pulse_iface snapshot (include/dpemu.h event record) */
            uint32_t *e = s->out->events + 4 * ((uint64_t)l->n_events * s->n_lanes + l->lane);
            e[0] = t;
            e[1] = (l->pr[0] & 0xFFFFFF) | ((l->pr[4] & 0xF) << 24) | (kind << 28);
            e[2] = (l->pr[1] & 0x1FFFF) | ((l->pr[2] & 0x1FF) << 17);
            e[3] = l->pr[3] & 0xFFFF;
        }
    } else l->flags |= DPEMU_F_EVENT_OVF;
    l->n_events++;

    const int demod = cfg->meas_model == DPEMU_MEAS_DEMOD;
    const uint32_t pp = (l->pr[1] & 0x1FFFF) | ((l->pr[2] & 0x1FF) << 17);
    if (demod) {                 /* the readout drive and the phase reference of the DEMOD model */
        if (kind == DPEMU_EV_PULSE_RESET) l->ro_tref = t;
        if (kind == DPEMU_EV_STROBE && (l->pr[4] & 3) == cfg->ro_drv_elem) {
            l->ro_d.have = 1; l->ro_d.t = t; l->ro_d.env = l->pr[0] & 0xFFFFFF;
            l->ro_d.pp = pp; l->ro_d.amp = l->pr[3] & 0xFFFF;
        }
    }
    /* measurement model: readout strobe -> meas_valid meas_latency clocks later
     * (DEMOD: after the readout window, in order) */
    if (kind == DPEMU_EV_STROBE && cfg->meas_elem != 0xFF && (l->pr[4] & 3) == cfg->meas_elem) {
        uint32_t core = l->core;
        uint32_t m = l->n_meas;
        uint32_t bit, tv;
        int32_t acc[2] = {0, 0};
        if (demod) {
            const uint32_t f_lo = oracle_ro_freq(l->ro_tab[1], l->ro_len[1], pp);
            const uint32_t f_d = oracle_ro_freq(l->ro_tab[0], l->ro_len[0], l->ro_d.pp);
            bit = oracle_demod(cfg, s->shot, core, m, t, l->pr[0] & 0xFFFFFF, pp, f_lo, &l->ro_d, f_d, l->ro_tref, acc);
            tv = oracle_demod_valid(cfg, t, l->pr[0] & 0xFFFFFF, l->ro_last_tv);
            l->ro_last_tv = tv;
        } else {
            bit = oracle_meas_bit(cfg->seed, s->shot, core, m, cfg->p1_threshold[core], l->pr[3],
                                  cfg->meas_model, cfg->ro_sep, cfg->ro_sigma, cfg->ro_thr,
                                  cfg->ro_win, l->pr[0]);
            tv = t + cfg->meas_latency;
        }
        if (m < MEAS_LOOKUP) { l->mt[m] = tv; l->mb[m] = (uint8_t)bit; }
        if (m < cfg->meas_cap) {
            if (s->out->meas) {
                uint32_t *e = s->out->meas + 2 * ((uint64_t)m * s->n_lanes + l->lane);
                e[0] = tv; e[1] = bit;
            }
            if (s->out->acc) {
                int32_t *e = s->out->acc + 2 * ((uint64_t)m * s->n_lanes + l->lane);
                e[0] = acc[0]; e[1] = acc[1];
            }
        } else l->flags |= DPEMU_F_MEAS_OVF;
        if (m >= MEAS_LOOKUP) l->flags |= DPEMU_F_MEAS_OVF;
        if (m < 32 && bit) l->meas_bits |= 1u << m;
        l->last_bit = bit;
        l->n_meas++;
    }
}

static void emit_trace(fshot *s, flane *l, uint32_t t, uint32_t addr, uint32_t val)
{
    if (l->n_trace < s->cfg->trace_cap) {
        if (s->out->trace) {
            uint32_t *e = s->out->trace + 4 * ((uint64_t)l->n_trace * s->n_lanes + l->lane);
            e[0] = t; e[1] = addr; e[2] = val; e[3] = 0;
        }
    } else if (s->cfg->trace_cap) l->flags |= DPEMU_F_TRACE_OVF;
    l->n_trace++;
}

static void finish(flane *l, uint32_t status, uint32_t t)
{
    l->status = status;
    l->mode = M_FIN;
    l->t_end = t;
    l->ip_end = l->ip;
    l->qclk_end = qclk_at(l, t);
}

/* latest measurement of lane q with valid cycle <= d (fproc_meas: meas_reg at d+1) */
static uint32_t meas_lookup(const flane *q, uint32_t d)
{
    uint32_t n = q->n_meas < MEAS_LOOKUP ? q->n_meas : MEAS_LOOKUP;
    for (uint32_t i = n; i-- > 0;)
        if (q->mt[i] <= d) return q->mb[i];
    return 0;
}

/* complete an fproc instruction of lane l decoded at D with ready cycle R, data */
static void fproc_complete(fshot *s, flane *l, const uint32_t w[4], uint32_t R, uint32_t data)
{
    uint32_t opcode = w[3] >> 24, op4 = opcode >> 4;
    uint32_t in0 = ((opcode >> 3) & 1) ? l->regs[fbits(w, 116, 4)] : fbits(w, 88, 32);
    uint32_t out = oracle_alu(opcode & 7, in0, data);
    if (op4 == 0x4) {
        uint32_t rd = fbits(w, 80, 4);
        l->regs[rd] = out;
        emit_trace(s, l, R + 3, rd, out);
        l->ip = (l->ip + 1) & 0xFFFF;
        l->t = R + 4;
    } else {
        l->ip = (out & 1) ? (fbits(w, 68, 16) & 0xFFFF) : ((l->ip + 1) & 0xFFFF);
        l->t = R + 6;
    }
    l->mode = M_RUN;
}

static void fetch(const flane *l, uint32_t w[4])
{
    if (l->ip < l->n_instr) memcpy(w, l->prog + 4 * (size_t)l->ip, 16);
    else memset(w, 0, 16);
}

static void sync_release(fshot *s, flane *l, uint32_t S)
{
    if (S > s->cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, l->wait_d); return; }
    l->qa_t = S + 2; l->qa_q = 0;
    emit_trace(s, l, S + 2, DPEMU_TRACE_QCLK_RST, 0);
    l->ip = (l->ip + 1) & 0xFFFF;
    l->t = S + 3;
    l->mode = M_RUN;
}

static void try_barrier(fshot *s)
{
    uint32_t maxd = 0;
    for (uint32_t c = 0; c < s->C; c++) {
        if (!((s->part >> c) & 1)) continue;
        if (s->L[c].mode != M_SYNC) return;
        if (s->L[c].wait_d > maxd) maxd = s->L[c].wait_d;
    }
    uint32_t S = maxd + s->cfg->sync_latency;
    for (uint32_t c = 0; c < s->C; c++)
        if ((s->part >> c) & 1) sync_release(s, &s->L[c], S);
}

/* ---- meas_lut evolution over the merged measurement stream ------------------ */
static void lut_apply_cycle(fshot *s, uint32_t tv, uint64_t valid, uint64_t meas)
{
    const dpemu_config *cfg = s->cfg;
    if (s->lut_ready_next && tv == s->lut_last_fire + 1) return;   /* LUT_READY: inputs ignored */
    uint64_t v = s->lut_valid | valid, a = s->lut_addr | (valid & meas);
    if ((cfg->lut_mask & v) == cfg->lut_mask) {
        s->lut_last_fire = tv; s->lut_ready_next = 1;
        if (s->nfire < LUT_FIRE_CAP) { s->fire_t[s->nfire] = tv; s->fire_out[s->nfire] = cfg->lut_table[a & 0xFF]; }
        s->nfire++;
        s->lut_valid = 0; s->lut_addr = 0;
    } else { s->lut_valid = v; s->lut_addr = a; }
}

/* apply every known measurement with valid cycle <= H, in time order;
 * stop_at_fire: stop after the first new fire (no-RUN-lane resolution) */
static void lut_advance(fshot *s, uint32_t H, int stop_at_fire)
{
    for (;;) {
        uint32_t tmin = INF32;
        for (uint32_t c = 0; c < s->C; c++) {
            flane *l = &s->L[c];
            uint32_t n = l->n_meas < MEAS_LOOKUP ? l->n_meas : MEAS_LOOKUP;
            if (s->lut_cursor[c] < n && l->mt[s->lut_cursor[c]] < tmin) tmin = l->mt[s->lut_cursor[c]];
        }
        if (tmin == INF32 || tmin > H) break;
        uint64_t valid = 0, meas = 0;
        for (uint32_t c = 0; c < s->C; c++) {
            flane *l = &s->L[c];
            uint32_t n = l->n_meas < MEAS_LOOKUP ? l->n_meas : MEAS_LOOKUP;
            if (s->lut_cursor[c] < n && l->mt[s->lut_cursor[c]] == tmin) {
                valid |= 1ull << c;
                if (l->mb[s->lut_cursor[c]]) meas |= 1ull << c;
                s->lut_cursor[c]++;
            }
        }
        uint32_t nf = s->nfire;
        lut_apply_cycle(s, tmin, valid, meas);
        if (stop_at_fire && s->nfire != nf) break;
    }
}

/* lower bound of any future readout strobe of lane l */
static uint32_t strobe_bound(const fshot *s, const flane *l)
{
    switch (l->mode) {
    case M_RUN: return l->t + 2;
    case M_LUT: return l->wait_d + 7;
    case M_SYNC: {
        if (!((s->part >> l->core) & 1)) return INF32;   /* never released */
        uint64_t m = 0;
        for (uint32_t c = 0; c < s->C; c++) {
            if (!((s->part >> c) & 1)) continue;
            const flane *p = &s->L[c];
            uint64_t v = (p->mode == M_SYNC) ? p->wait_d : (p->mode == M_RUN) ? p->t
                       : (p->mode == M_LUT) ? (uint64_t)p->wait_d + 5 : (uint64_t)INF32;
            if (v > m) m = v;
        }
        m += s->cfg->sync_latency + 5;
        return m > INF32 ? INF32 : (uint32_t)m;
    }
    default: return INF32;
    }
}

static int lut_resolve(fshot *s)
{
    int progressed = 0;
    for (uint32_t c = 0; c < s->C; c++) {
        flane *l = &s->L[c];
        if (l->mode != M_LUT) continue;
        for (uint32_t k = 0; k < s->nfire && k < LUT_FIRE_CAP; k++) {
            if (s->fire_t[k] >= l->wait_d + 1) {
                uint32_t R = s->fire_t[k];
                if (R > s->cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, l->wait_d); }
                else {
                    uint32_t w[4]; fetch(l, w);
                    fproc_complete(s, l, w, R, (uint32_t)((s->fire_out[k] >> c) & 1));
                }
                progressed = 1;
                break;
            }
        }
    }
    return progressed;
}

static void lut_step(fshot *s, int any_run)
{
    if (any_run) {
        uint32_t H = INF32;
        for (uint32_t c = 0; c < s->C; c++) {
            uint32_t b = strobe_bound(s, &s->L[c]);
            if (b != INF32) {
                uint64_t h = (uint64_t)b + s->cfg->meas_latency - 1;
                if (h < H) H = (uint32_t)h;
            }
        }
        lut_advance(s, H, 0);
    }
    lut_resolve(s);
}

/* execute the instruction of lane l at its DECODE cycle l->t */
static void exec_one(fshot *s, flane *l)
{
    const dpemu_config *cfg = s->cfg;
    uint32_t D = l->t;
    if (D > cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, D); return; }
    uint32_t w[4];
    fetch(l, w);
    uint32_t opcode = w[3] >> 24, op4 = opcode >> 4, alu_op = opcode & 7;
    uint32_t in0 = ((opcode >> 3) & 1) ? l->regs[fbits(w, 116, 4)] : fbits(w, 88, 32);
    uint32_t qD = qclk_at(l, D);
    l->n_instr_exec++;
    switch (op4) {
    case 0x0: case 0xA:
        finish(l, DPEMU_ST_DONE, D);
        return;
    case 0xD: case 0xE: case 0xF:
        finish(l, DPEMU_ST_HUNG_OPCODE, D);
        return;
    case 0x8:
        oracle_pulse_reg(l->pr, w, l->regs[fbits(w, 116, 4)], 1);
        l->ip = (l->ip + 1) & 0xFFFF; l->t = D + 3;
        return;
    case 0xB:
        emit_event(s, l, D, DPEMU_EV_PULSE_RESET);
        l->ip = (l->ip + 1) & 0xFFFF; l->t = D + 3;
        return;
    case 0x9: case 0xC: {
        uint32_t T = fbits(w, 5, 32);
        uint64_t tT; int dbl = 0;
        if (D < l->qa_t) {                        /* reset hold: qclk(0) = qclk(1) = 0 */
            if (T == 0) { tT = D; dbl = 1; }
            else tT = (uint64_t)l->qa_t + (uint32_t)(T - l->qa_q);
        } else tT = (uint64_t)D + (uint32_t)(T - qD);
        if (tT - D >= 0x80000000ull) l->flags |= DPEMU_F_LATE;
        if (tT > cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, D); return; }
        if (op4 == 0x9) {
            oracle_pulse_reg(l->pr, w, l->regs[fbits(w, 116, 4)], 1);
            emit_event(s, l, (uint32_t)tT + 2, DPEMU_EV_STROBE);
            if (dbl) { emit_event(s, l, (uint32_t)tT + 3, DPEMU_EV_STROBE); l->flags |= DPEMU_F_DOUBLE_STROBE; }
        }
        l->ip = (l->ip + 1) & 0xFFFF; l->t = (uint32_t)tT + 3;
        return;
    }
    case 0x1: {
        uint32_t out = oracle_alu(alu_op, in0, l->regs[fbits(w, 84, 4)]);
        uint32_t rd = fbits(w, 80, 4);
        l->regs[rd] = out;
        emit_trace(s, l, D + 3, rd, out);
        l->ip = (l->ip + 1) & 0xFFFF; l->t = D + 4;
        return;
    }
    case 0x2:
        l->ip = fbits(w, 68, 16) & 0xFFFF; l->t = D + 4;
        return;
    case 0x3: {
        uint32_t out = oracle_alu(alu_op, in0, l->regs[fbits(w, 84, 4)]);
        l->ip = (out & 1) ? (fbits(w, 68, 16) & 0xFFFF) : ((l->ip + 1) & 0xFFFF);
        l->t = D + 6;
        return;
    }
    case 0x6: {
        uint32_t out = oracle_alu(alu_op, in0, qD);
        l->qa_t = D + 3; l->qa_q = out + 3;
        emit_trace(s, l, D + 3, DPEMU_TRACE_QCLK_LOAD, out + 3);
        l->ip = (l->ip + 1) & 0xFFFF; l->t = D + 4;
        return;
    }
    case 0x4: case 0x5: {
        uint32_t id = fbits(w, 52, 8);
        if (cfg->fproc_mode == DPEMU_FPROC_MEAS) {
            uint32_t R = D + 2;
            if (R > cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, D); return; }
            uint32_t data = meas_lookup(&s->L[id & s->addr_mask], D);
            fproc_complete(s, l, w, R, data);
            return;
        }
        if (id == 0) {                           /* core_state_mgr WAIT_MEAS: own next meas_valid */
            uint32_t n = l->n_meas < MEAS_LOOKUP ? l->n_meas : MEAS_LOOKUP;
            for (uint32_t i = 0; i < n; i++) {
                if (l->mt[i] >= D + 1) {
                    if (l->mt[i] > cfg->max_cycles) { finish(l, DPEMU_ST_MAX_CYCLES, D); return; }
                    fproc_complete(s, l, w, l->mt[i], l->mb[i]);
                    return;
                }
            }
            finish(l, DPEMU_ST_DEADLOCK, D);
            return;
        }
        l->mode = M_LUT; l->wait_d = D;          /* WAIT_LUT */
        return;
    }
    case 0x7:
        /* a core outside sync_mask never receives ready: it waits forever */
        l->mode = M_SYNC; l->wait_d = D;
        try_barrier(s);
        return;
    default:
        return;
    }
}

static void run_shot(fshot *s)
{
    const uint32_t C = s->C;
    for (;;) {
        flane *best = NULL;
        for (uint32_t c = 0; c < C; c++) {
            flane *l = &s->L[c];
            if (l->mode == M_RUN && (!best || l->t < best->t)) best = l;
        }
        if (best) {
            exec_one(s, best);
            if (s->cfg->fproc_mode == DPEMU_FPROC_LUT) lut_step(s, 1);
            continue;
        }
        /* no core can run: LUT fires from the known measurements may still release one */
        int waiting = 0;
        for (uint32_t c = 0; c < C; c++) if (s->L[c].mode == M_LUT || s->L[c].mode == M_SYNC) waiting = 1;
        if (!waiting) break;
        if (s->cfg->fproc_mode == DPEMU_FPROC_LUT) {
            uint32_t nf = s->nfire;
            lut_advance(s, INF32, 1);
            if (lut_resolve(s) || s->nfire != nf) continue;
        }
        for (uint32_t c = 0; c < C; c++)
            if (s->L[c].mode == M_LUT || s->L[c].mode == M_SYNC) finish(&s->L[c], DPEMU_ST_DEADLOCK, s->L[c].wait_d);
    }
}

int fast_run(const dpemu_config *cfg, const uint32_t *words, const uint32_t *offsets,
             const uint32_t *n_instr, const uint32_t *prog_table, uint64_t shot_begin,
             uint64_t n_shots, const dpemu_outputs *out, int n_threads,
             const uint32_t *ro_words, const uint32_t *ro_hdr)
{
    const uint32_t C = cfg->cores_per_shot;
    if (C == 0 || C > DPEMU_MAX_CORES || (C & (C - 1))) return DPEMU_E_INVALID;
    const uint64_t n_lanes = n_shots * C;
    uint32_t hist_bins = (C <= 12) ? (1u << C) : 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    #pragma omp parallel for schedule(dynamic, 64)
    for (int64_t si = 0; si < (int64_t)n_shots; si++) {
        fshot *s = (fshot *)malloc(sizeof(fshot));
        memset(s, 0, offsetof(fshot, L));
        uint64_t shot = shot_begin + (uint64_t)si;
        s->cfg = cfg; s->out = out; s->n_lanes = n_lanes; s->shot = shot; s->C = C;
        s->addr_mask = C - 1;
        uint64_t all = (C >= 64) ? ~0ull : ((1ull << C) - 1);
        s->part = cfg->sync_mask ? (cfg->sync_mask & all) : all;
        uint32_t g = (uint32_t)((shot / cfg->shots_per_group) % cfg->n_groups);
        for (uint32_t c = 0; c < C; c++) {
            flane *l = &s->L[c];
            memset(l, 0, sizeof(*l));
            uint32_t p = prog_table[(uint64_t)g * C + c];
            l->prog = words + 4 * (uint64_t)offsets[p];
            l->n_instr = n_instr[p];
            l->qa_t = 1; l->qa_q = 0;
            l->lane = cfg->lane_order == DPEMU_LANES_SHOT_MAJOR      /* include/dpemu.h lane order */
                          ? (uint32_t)((uint64_t)si * C + c) : (uint32_t)((uint64_t)c * n_shots + (uint64_t)si);
            l->core = c;
            if (ro_words && ro_hdr) {
                const uint32_t *h = ro_hdr + 4 * (uint64_t)p;
                l->ro_tab[0] = ro_words + h[0]; l->ro_len[0] = h[1];
                l->ro_tab[1] = ro_words + h[2]; l->ro_len[1] = h[3];
            }
        }
        run_shot(s);
        uint32_t key = 0;
        for (uint32_t c = 0; c < C; c++) {
            flane *l = &s->L[c];
            if (out->summary) {
                uint32_t *sm = out->summary + 8 * (uint64_t)l->lane;
                sm[0] = l->t_end;
                sm[1] = (l->ip_end & 0xFFFF) | ((l->status & 0xFF) << 16) | ((l->flags & 0xFF) << 24);
                sm[2] = l->n_events; sm[3] = l->n_instr_exec; sm[4] = l->qclk_end;
                sm[5] = l->n_meas; sm[6] = l->meas_bits; sm[7] = l->n_trace;
            }
            if (out->regs)
                for (int r = 0; r < 16; r++) out->regs[(uint64_t)r * n_lanes + l->lane] = l->regs[r];
            if (l->last_bit) key |= 1u << c;
        }
        if (out->hist && hist_bins) {
            #pragma omp atomic
            out->hist[(uint64_t)g * hist_bins + key] += 1;
        }
        free(s);
    }
    return DPEMU_OK;
}
