/*
 * oracle/rtl_model.c -- TEST INFRASTRUCTURE (oracle_rtl).
 *
 * Literal per-clock restatement of the reference gateware, evaluated the way
 * a cycle simulator evaluates it: every call to rtl_shot_step() computes the
 * combinational logic of one clock from the current register values and
 * inputs, then commits every register (non-blocking semantics).
 *
 *   rtl_core   one proc (hdl/proc.sv:9-171) with its toplevel_sim cmd_mem
 *              (sim_modules/toplevel_sim.sv:69-76, 4 x 32-bit banks,
 *              READ_LATENCY 3) -- ctrl.v, alu.v, instr_ptr.v, qclk.v,
 *              reg_file.v, cmd_mem.v, pulse_reg.sv each restated below.
 *   rtl_shot   C cores + the shared fproc back end (fproc_meas.sv or
 *              fproc_lut.sv = core_state_mgr.sv + meas_lut.sv), the
 *              build-defined sync controller and measurement model
 *               -- or "external" inputs so the cocotb
 *              testbenches can drive fproc/sync themselves.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this file, as the checker.  It is never part of the product path.
 */
#include "oracle.h"

#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <string.h>

#define T0 6u   /* clocks from the start of reset to the first DECODE (rtl_run_shot) */

/* ctrl.v:84-91 */
enum { S_MEM_WAIT = 0, S_DECODE = 1, S_ALU0 = 2, S_ALU1 = 3, S_FPROC_WAIT = 4,
       S_SYNC_WAIT = 6, S_QCLK_RST = 7, S_DONE = 9 };

/* ---------------------------------------------------------------------- */
/* field slicing of the 128-bit local_cmd (proc.sv:89-107)                 */
/* ---------------------------------------------------------------------- */
static uint32_t bits128(const uint32_t w[4], int lo, int width)
{
    /* width <= 32 */
    uint64_t acc = 0;
    int word = lo >> 5, off = lo & 31;
    acc = w[word];
    if (word < 3) acc |= (uint64_t)w[word + 1] << 32;
    acc >>= off;
    return (uint32_t)(acc & ((width == 32) ? 0xFFFFFFFFull : ((1ull << width) - 1)));
}

/* alu.v: registered inputs, combinational op, registered output */
uint32_t oracle_alu(uint32_t ctrl, uint32_t in0, uint32_t in1)
{
    uint32_t sub = in0 - in1;
    uint32_t s0 = in0 >> 31, s1 = in1 >> 31, ss = sub >> 31;
    uint32_t oflow = ((!s0) & s1 & ss) | (s0 & (!s1) & (!ss));
    uint32_t le = ss ^ oflow;
    switch (ctrl & 7) {
    case 0: return in0;
    case 1: return in0 + in1;
    case 2: return sub;
    case 3: return sub == 0;
    case 4: return le;
    case 5: return !le;
    case 6: return in1;
    default: return 0;
    }
}

/* pulse_reg.sv:59-97: next {env, phase, freq, amp, cfg} for pulse_cmd_in =
 * cmd[115:37] (proc.sv:103), reg_in = reg[cmd[119:116]] (proc.sv:156) */
void oracle_pulse_reg(uint32_t pr[5], const uint32_t lc[4], uint32_t reg_in, int write_en)
{
    if (!write_en) return;
    if (bits128(lc, 115, 1)) pr[0] = bits128(lc, 114, 1) ? (reg_in & 0xFFFFFF) : bits128(lc, 90, 24);
    if (bits128(lc, 89, 1))  pr[1] = bits128(lc, 88, 1) ? (reg_in & 0x1FFFF) : bits128(lc, 71, 17);
    if (bits128(lc, 70, 1))  pr[2] = bits128(lc, 69, 1) ? (reg_in & 0x1FF) : bits128(lc, 60, 9);
    if (bits128(lc, 59, 1))  pr[3] = bits128(lc, 58, 1) ? (reg_in & 0xFFFF) : bits128(lc, 42, 16);
    if (bits128(lc, 41, 1))  pr[4] = bits128(lc, 37, 4);
}

/* ctrl.v:163-593: combinational outputs of the FSM */
typedef struct {
    int next_state, mem_wait_rst, ip_en, load_en, ip_load_sel, in1_sel;
    int reg_we, qclk_load, qclk_rst, cstrobe_en, trig_en, pulse_we, done_gate;
    int pulse_reset, sync_en, fproc_en;
} ctrl_out;

static void ctrl_eval(int state, uint32_t mwc, uint32_t opcode, int fproc_ready, int sync_ready,
                      int trig_in, ctrl_out *o)
{
    int op4 = (opcode >> 4) & 0xF;
    memset(o, 0, sizeof(*o));
    o->in1_sel = 1;            /* ALU_IN1_REG_SEL is the default everywhere */
    switch (state) {
    case S_MEM_WAIT:
        if (mwc < 2) { o->next_state = S_MEM_WAIT; }
        else { o->load_en = 1; o->mem_wait_rst = 1; o->ip_en = 1; o->next_state = S_DECODE; }
        break;
    case S_DECODE:
        switch (op4) {
        case 0x8: o->next_state = S_MEM_WAIT; o->pulse_we = 1; break;
        case 0x9: o->next_state = trig_in ? S_MEM_WAIT : S_DECODE;
                  o->cstrobe_en = 1; o->trig_en = 1; o->pulse_we = 1; break;
        case 0xC: o->next_state = trig_in ? S_MEM_WAIT : S_DECODE; o->trig_en = 1; break;
        case 0xB: o->next_state = S_MEM_WAIT; o->pulse_reset = 1; break;
        case 0x1: case 0x3: o->next_state = S_ALU0; break;
        case 0x6: o->next_state = S_ALU0; o->in1_sel = 0; break;     /* QCLK_SEL */
        case 0x2: o->next_state = S_MEM_WAIT; o->mem_wait_rst = 1; o->ip_load_sel = 1; break;
        case 0x4: case 0x5: o->next_state = S_FPROC_WAIT; o->fproc_en = 1; break;
        case 0x7: o->next_state = S_SYNC_WAIT; o->sync_en = 1; break;
        case 0xA: case 0x0: o->next_state = S_DONE; o->mem_wait_rst = 1; break;
        default:  o->next_state = S_DECODE; break;                   /* hang */
        }
        break;
    case S_ALU0:
        o->next_state = S_ALU1;
        break;
    case S_ALU1:
        o->next_state = S_MEM_WAIT;
        switch (op4) {
        case 0x1: case 0x4: o->reg_we = 1; break;
        case 0x3: case 0x5: o->mem_wait_rst = 1; o->ip_load_sel = 2; break;  /* LOAD_EN_ALU */
        case 0x6: o->qclk_load = 1; break;
        default: break;
        }
        break;
    case S_FPROC_WAIT:
        o->next_state = fproc_ready ? S_ALU0 : S_FPROC_WAIT;
        o->in1_sel = 2;
        break;
    case S_SYNC_WAIT:
        o->next_state = sync_ready ? S_QCLK_RST : S_SYNC_WAIT;
        o->in1_sel = 2;
        break;
    case S_QCLK_RST:
        o->next_state = S_MEM_WAIT; o->in1_sel = 0; o->qclk_rst = 1;
        break;
    case S_DONE:
        o->next_state = S_DONE; o->done_gate = 1;
        break;
    default:
        o->next_state = S_MEM_WAIT;
        break;
    }
}

/* ---------------------------------------------------------------------- */
/* one proc core                                                           */
/* ---------------------------------------------------------------------- */
void rtl_core_init(rtl_core *c, const uint32_t *prog, uint32_t n_instr, int addr_width)
{
    memset(c, 0, sizeof(*c));   /* Verilator zero-initialises every register */
    c->prog = prog;
    c->n_instr = n_instr;
    c->addr_mask = (addr_width >= 32) ? 0xFFFFFFFFu : ((1u << addr_width) - 1);
}

static void fetch_word(const rtl_core *c, uint32_t addr, uint32_t out[4])
{
    if (addr < c->n_instr) memcpy(out, c->prog + 4 * (size_t)addr, 16);
    else memset(out, 0, 16);
}

/* combinational half of one clock; fills c->comb and c->nxt (next register values) */
void rtl_core_eval(rtl_core *c, int reset, int fproc_ready, uint32_t fproc_data, int sync_ready)
{
    rtl_core_comb *o = &c->comb;
    const uint32_t *lc = c->lc;
    uint32_t opcode = lc[3] >> 24;
    ctrl_out k;
    ctrl_eval(c->state, c->mwc, opcode, fproc_ready, sync_ready, c->qclk_trig, &k);

    uint32_t alu_op = opcode & 7, in0_sel = (opcode >> 3) & 1;
    uint32_t rs0 = bits128(lc, 116, 4), rs1 = bits128(lc, 84, 4), rd = bits128(lc, 80, 4);
    uint32_t imm = bits128(lc, 88, 32);
    uint32_t target = bits128(lc, 68, 16) & c->addr_mask;
    uint32_t cmd_time = bits128(lc, 5, 32);
    uint32_t reg0 = c->regs[rs0], reg1 = c->regs[rs1];
    uint32_t alu_in0 = in0_sel ? reg0 : imm;
    uint32_t alu_in1 = (k.in1_sel & 2) ? fproc_data : ((k.in1_sel & 1) ? reg1 : c->qclk);
    int ip_load = (k.ip_load_sel & 2) ? (int)(c->alu_out & 1) : (k.ip_load_sel & 1);
    uint32_t cur_ip = ip_load ? target : (k.ip_en ? c->ipv_inc : c->ipv);
    cur_ip &= c->addr_mask;
    uint32_t cmd_buf_out[4];
    fetch_word(c, c->ra[2], cmd_buf_out);
    int qclk_reset = k.qclk_rst || (c->reset_sr & 0xF);

    /* observable outputs of this cycle */
    o->state = c->state;
    o->opcode = opcode;
    o->qclk = c->qclk;
    o->cstrobe = c->p_cstrobe;
    o->env = c->p_env; o->phase = c->p_phase; o->freq = c->p_freq;
    o->amp = c->p_amp; o->cfg = c->p_cfg;
    o->pulse_reset = k.pulse_reset;
    o->done_gate = k.done_gate;
    o->sync_enable = k.sync_en;
    o->fproc_enable = k.fproc_en;
    o->fproc_id = bits128(lc, 52, 8);
    o->instr_ptr = cur_ip;
    o->load_en = k.load_en;
    o->load_addr = c->ra[2];
    memcpy(o->cmd_buf_out, cmd_buf_out, 16);
    o->reg_we = k.reg_we; o->reg_wa = rd; o->reg_wd = c->alu_out;
    o->qclk_load = k.qclk_load; o->qclk_rst_ctrl = k.qclk_rst;

    /* next register values */
    rtl_core_regs *n = &c->nxt;
    n->reset_reg = (uint8_t)reset;
    n->reset_sr = (uint8_t)(((c->reset_sr << 1) | c->reset_reg) & 0x1F);
    n->qclk_trig = (uint8_t)((c->qclk == cmd_time) && k.trig_en);
    n->cstrobe_p = (uint8_t)((c->qclk == cmd_time) && k.cstrobe_en);
    if (c->reset_reg) { n->state = S_MEM_WAIT; n->mwc = 0; }
    else { n->state = k.next_state; n->mwc = k.mem_wait_rst ? 0 : c->mwc + 1; }
    if (k.load_en) memcpy(n->lc, cmd_buf_out, 16); else memcpy(n->lc, lc, 16);
    if (c->reset_reg) { n->ipv_inc = 1; n->ipv = 0; }
    else { n->ipv_inc = (cur_ip + 1) & c->addr_mask; n->ipv = cur_ip; }
    n->ra[0] = cur_ip; n->ra[1] = c->ra[0]; n->ra[2] = c->ra[1];
    n->alu_in0 = alu_in0; n->alu_in1 = alu_in1;
    n->alu_out = oracle_alu(alu_op, c->alu_in0, c->alu_in1);
    n->qclk = qclk_reset ? 0 : (k.qclk_load ? c->alu_out + 3 : c->qclk + 1);

    /* pulse_reg.sv:59-97 */
    uint32_t pr[5] = {c->p_env, c->p_phase, c->p_freq, c->p_amp, c->p_cfg};
    oracle_pulse_reg(pr, lc, reg0, k.pulse_we);
    n->p_env = pr[0]; n->p_phase = pr[1]; n->p_freq = pr[2]; n->p_amp = pr[3]; n->p_cfg = pr[4];
    n->p_cstrobe = c->cstrobe_p;
    n->reg_we = k.reg_we; n->reg_wa = rd; n->reg_wd = c->alu_out;
}

void rtl_core_commit(rtl_core *c)
{
    const rtl_core_regs *n = &c->nxt;
    c->reset_reg = n->reset_reg; c->reset_sr = n->reset_sr;
    c->qclk_trig = n->qclk_trig; c->cstrobe_p = n->cstrobe_p;
    c->state = n->state; c->mwc = n->mwc;
    memcpy(c->lc, n->lc, 16);
    c->ipv = n->ipv; c->ipv_inc = n->ipv_inc;
    memcpy(c->ra, n->ra, sizeof(c->ra));
    c->alu_in0 = n->alu_in0; c->alu_in1 = n->alu_in1; c->alu_out = n->alu_out;
    c->qclk = n->qclk;
    c->p_env = n->p_env; c->p_phase = n->p_phase; c->p_freq = n->p_freq;
    c->p_amp = n->p_amp; c->p_cfg = n->p_cfg; c->p_cstrobe = n->p_cstrobe;
    if (n->reg_we) c->regs[n->reg_wa] = n->reg_wd;
}

/* ---------------------------------------------------------------------- */
/* shared fproc back end                                                   */
/* ---------------------------------------------------------------------- */
static uint32_t clog2_mask(uint32_t n)
{
    uint32_t b = 0;
    while ((1u << b) < n) b++;
    return (b == 0) ? 0u : ((1u << b) - 1);
}

void rtl_fproc_init(rtl_fproc *f, uint32_t mode, uint32_t n, uint32_t lut_mask, const uint64_t *lut_table)
{
    memset(f, 0, sizeof(*f));
    f->mode = mode; f->n = n;
    f->addr_mask = clog2_mask(n);      /* fproc_meas.sv:12,27: id[$clog2(N_MEAS)-1:0] */
    f->lut_mask = lut_mask;
    if (lut_table) memcpy(f->lut_table, lut_table, sizeof(f->lut_table));
}

/* outputs of this clock: registered (fproc_meas) or combinational on meas inputs (fproc_lut) */
void rtl_fproc_eval(rtl_fproc *f, uint64_t valid, uint64_t meas)
{
    if (f->mode == DPEMU_FPROC_MEAS) {
        for (uint32_t c = 0; c < f->n; c++) { f->out_ready[c] = f->ready[c]; f->out_data[c] = f->data[c]; }
        return;
    }
    /* meas_lut.sv:27-56 */
    if (f->lut_state == 0) {
        f->lut_v = f->lut_valid | valid;
        f->lut_a = f->lut_addr | (valid & meas);
        f->lut_ready = ((f->lut_mask & f->lut_v) == f->lut_mask);
    } else {
        f->lut_v = 0; f->lut_a = 0;
        f->lut_ready = (f->lut_mask == 0);
    }
    uint64_t lut_out = f->lut_table[f->lut_a & 0xFF];
    /* core_state_mgr.sv:30-75 */
    for (uint32_t c = 0; c < f->n; c++) {
        f->out_ready[c] = 0; f->out_data[c] = 0;
        if (f->cs[c] == 1 && ((valid >> c) & 1)) { f->out_ready[c] = 1; f->out_data[c] = (uint32_t)((meas >> c) & 1); }
        if (f->cs[c] == 2 && f->lut_ready) { f->out_ready[c] = 1; f->out_data[c] = (uint32_t)((lut_out >> c) & 1); }
    }
}

void rtl_fproc_commit(rtl_fproc *f, int reset, uint64_t valid, uint64_t meas,
                      const uint32_t *enable, const uint32_t *id)
{
    if (f->mode == DPEMU_FPROC_MEAS) {
        /* fproc_meas.sv:18-34 (its reset input is unused) */
        uint64_t mr = f->meas_reg;
        for (uint32_t c = 0; c < f->n; c++) {
            f->ready[c] = f->arm[c];
            f->data[c] = (uint32_t)((mr >> f->addr[c]) & 1);
            f->arm[c] = (uint8_t)(enable[c] != 0);
            f->addr[c] = id[c] & f->addr_mask;
        }
        f->meas_reg = (mr & ~valid) | (meas & valid);
        return;
    }
    for (uint32_t c = 0; c < f->n; c++) {
        uint8_t st = f->cs[c];
        if (reset) f->cs[c] = 0;
        else if (st == 0) f->cs[c] = enable[c] ? (id[c] == 0 ? 1 : 2) : 0;
        else if (st == 1) f->cs[c] = ((valid >> c) & 1) ? 0 : 1;
        else f->cs[c] = f->lut_ready ? 0 : 2;
    }
    if (reset) { f->lut_state = 0; f->lut_valid = 0; f->lut_addr = 0; }
    else if (f->lut_state == 0) {
        if (f->lut_ready) { f->lut_state = 1; f->lut_valid = 0; f->lut_addr = 0; }
        else { f->lut_valid = f->lut_v; f->lut_addr = f->lut_a; }
    } else { f->lut_state = 0; f->lut_valid = 0; f->lut_addr = 0; }
}

/* ---------------------------------------------------------------------- */
/* a shot: C cores + shared fproc + sync controller + measurement model     */
/* ---------------------------------------------------------------------- */
void rtl_shot_init(rtl_shot *s, const oracle_shot_cfg *cfg, const uint32_t *const *progs,
                   const uint32_t *n_instr, uint64_t shot_index)
{
    memset(s, 0, sizeof(*s));
    s->cfg = *cfg;
    s->shot = shot_index;
    for (uint32_t c = 0; c < cfg->cores; c++)
        rtl_core_init(&s->core[c], progs[c], n_instr[c], 16);
    rtl_fproc_init(&s->fp, cfg->fproc_mode == ORACLE_FPROC_EXTERNAL ? DPEMU_FPROC_MEAS : cfg->fproc_mode,
                   cfg->cores, cfg->lut_mask, cfg->lut_table);
    s->sync_mask = cfg->sync_mask ? cfg->sync_mask
                                  : ((cfg->cores >= 64) ? ~0ull : ((1ull << cfg->cores) - 1));
}

/* meas_valid / meas inputs of this cycle, from the scheduled readouts */
static void meas_inputs(rtl_shot *s, uint64_t *valid, uint64_t *meas)
{
    *valid = 0; *meas = 0;
    for (uint32_t c = 0; c < s->cfg.cores; c++) {
        rtl_meas_q *q = &s->mq[c];
        if (q->head < q->tail && q->t[q->head % RTL_MQ] == s->cycle) {
            *valid |= 1ull << c;
            if (q->bit[q->head % RTL_MQ]) *meas |= 1ull << c;
        }
    }
}

void rtl_shot_step(rtl_shot *s, const rtl_ext_inputs *ext)
{
    const uint32_t C = s->cfg.cores;
    int reset = ext ? ext->reset : (s->cycle < 2);
    uint64_t valid = 0, meas = 0;
    if (ext && ext->drive_meas) { valid = ext->meas_valid; meas = ext->meas; }
    else meas_inputs(s, &valid, &meas);
    s->cur_valid = valid; s->cur_meas = meas;

    int fready[DPEMU_MAX_CORES]; uint32_t fdata[DPEMU_MAX_CORES];
    if (s->cfg.fproc_mode == ORACLE_FPROC_EXTERNAL) {
        for (uint32_t c = 0; c < C; c++) { fready[c] = ext->fproc_ready[c]; fdata[c] = ext->fproc_data[c]; }
    } else {
        rtl_fproc_eval(&s->fp, valid, meas);
        for (uint32_t c = 0; c < C; c++) { fready[c] = s->fp.out_ready[c]; fdata[c] = s->fp.out_data[c]; }
    }
    int sready = s->cfg.sync_external ? ext->sync_ready : (s->sync_pend && s->sync_t == s->cycle);

    /* the controller drives ready to the barrier's participants only */
    for (uint32_t c = 0; c < C; c++)
        rtl_core_eval(&s->core[c], reset, fready[c], fdata[c],
                      sready && (s->cfg.sync_external || ((s->sync_mask >> c) & 1)));

    /* measurement model: a readout strobe schedules meas_valid latency clocks
     * later (DEMOD: after its window, in order; oracle/readout.c) */
    const int demod = s->cfg.meas_model == DPEMU_MEAS_DEMOD;
    for (uint32_t c = 0; c < C; c++) {
        const rtl_core_comb *o = &s->core[c].comb;
        const uint32_t tnow = (uint32_t)(s->cycle - T0);      /* dpemu time of this clock */
        if (demod && s->cycle >= T0) {
            if (o->pulse_reset) s->ro_tref[c] = tnow;
            if (o->cstrobe && (o->cfg & 3) == s->cfg.ro.ro_drv_elem) {
                oracle_ro_drive *d = &s->ro_d[c];
                d->have = 1; d->t = tnow; d->env = o->env & 0xFFFFFF;
                d->pp = (o->phase & 0x1FFFF) | ((o->freq & 0x1FF) << 17); d->amp = o->amp & 0xFFFF;
            }
        }
        if (o->cstrobe && s->cfg.meas_elem != 0xFF && (o->cfg & 3) == s->cfg.meas_elem) {
            uint32_t m = s->n_meas[c]++;
            rtl_meas_q *q = &s->mq[c];
            int bit;
            if (demod) {
                const uint32_t pp = (o->phase & 0x1FFFF) | ((o->freq & 0x1FF) << 17);
                const uint32_t f_lo = oracle_ro_freq(s->cfg.ro_tab[c][1], s->cfg.ro_len[c][1], pp);
                const uint32_t f_d = oracle_ro_freq(s->cfg.ro_tab[c][0], s->cfg.ro_len[c][0], s->ro_d[c].pp);
                bit = (int)oracle_demod(&s->cfg.ro, s->shot, c, m, tnow, o->env & 0xFFFFFF, pp, f_lo, &s->ro_d[c],
                                        f_d, s->ro_tref[c], s->ro_acc[c][q->tail % RTL_MQ]);
                const uint32_t tv = oracle_demod_valid(&s->cfg.ro, tnow, o->env & 0xFFFFFF,
                                                       (uint32_t)s->ro_last_tv[c]);
                s->ro_last_tv[c] = tv;
                q->t[q->tail % RTL_MQ] = (uint64_t)tv + T0;
            } else {
                bit = (int)oracle_meas_bit(s->cfg.seed, s->shot, c, m, s->cfg.p1_threshold[c], o->amp,
                                           s->cfg.meas_model, s->cfg.ro_sep, s->cfg.ro_sigma, s->cfg.ro_thr,
                                           s->cfg.ro_win, o->env);
                q->t[q->tail % RTL_MQ] = s->cycle + s->cfg.meas_latency;
            }
            q->bit[q->tail % RTL_MQ] = (uint8_t)bit;
            q->tail++;
        }
        if ((valid >> c) & 1) s->mq[c].head++;
    }

    if (s->cfg.fproc_mode != ORACLE_FPROC_EXTERNAL) {
        uint32_t en[DPEMU_MAX_CORES] = {0}, id[DPEMU_MAX_CORES] = {0};
        for (uint32_t c = 0; c < C; c++) { en[c] = s->core[c].comb.fproc_enable; id[c] = s->core[c].comb.fproc_id; }
        rtl_fproc_commit(&s->fp, reset, valid, meas, en, id);
    }

    /* sync controller (build-defined): ready to the participants `sync_latency`
     * clocks after the last participant's enable; then the next barrier begins */
    if (!s->cfg.sync_external) {
        uint64_t en = 0;
        for (uint32_t c = 0; c < C; c++) if (s->core[c].comb.sync_enable) en |= 1ull << c;
        if (s->sync_pend && s->sync_t == s->cycle) s->sync_pend = 0;
        uint64_t arr = s->sync_arrived | en;
        if (!s->sync_pend && (arr & s->sync_mask) == s->sync_mask) {
            s->sync_pend = 1;
            s->sync_t = s->cycle + s->cfg.sync_latency;
            arr = 0;
        }
        s->sync_arrived = arr;
    }

    for (uint32_t c = 0; c < C; c++) rtl_core_commit(&s->core[c]);
    s->cycle++;
}

/* ---------------------------------------------------------------------- */
/* cocotb-style testbenches: inputs set before an edge apply to that cycle; */
/* values read after the edge are the ones of the cycle just clocked        */
/* ---------------------------------------------------------------------- */
struct rtl_tb {
    rtl_core core;
    uint32_t mem[65536 * 4];
    int reset, fproc_ready, sync_ready; uint32_t fproc_data;
    int wr_en; uint32_t wr_addr, wr_word[4];
    rtl_core_comb snap;
    uint32_t snap_regs[16];
    uint64_t cycle;
};

rtl_tb *rtl_tb_new(void)
{
    rtl_tb *tb = (rtl_tb *)calloc(1, sizeof(rtl_tb));
    rtl_core_init(&tb->core, tb->mem, 65536, 16);
    return tb;
}

void rtl_tb_free(rtl_tb *tb) { free(tb); }

void rtl_tb_set(rtl_tb *tb, int reset, int fproc_ready, uint32_t fproc_data, int sync_ready)
{
    tb->reset = reset; tb->fproc_ready = fproc_ready; tb->fproc_data = fproc_data; tb->sync_ready = sync_ready;
}

void rtl_tb_write(rtl_tb *tb, int en, uint32_t addr, const uint32_t *word)
{
    tb->wr_en = en; tb->wr_addr = addr & 0xFFFF;
    if (word) memcpy(tb->wr_word, word, 16);
}

void rtl_tb_edge(rtl_tb *tb)
{
    rtl_core_eval(&tb->core, tb->reset, tb->fproc_ready, tb->fproc_data, tb->sync_ready);
    tb->snap = tb->core.comb;
    memcpy(tb->snap_regs, tb->core.regs, sizeof(tb->snap_regs));
    rtl_core_commit(&tb->core);
    if (tb->wr_en) memcpy(tb->mem + 4 * (size_t)tb->wr_addr, tb->wr_word, 16);   /* cmd_mem.v:19-20 */
    tb->cycle++;
}

const rtl_core_comb *rtl_tb_snap(const rtl_tb *tb) { return &tb->snap; }
uint32_t rtl_tb_reg(const rtl_tb *tb, int i) { return tb->snap_regs[i & 15]; }

struct rtl_fproc_tb { rtl_fproc f; int reset; uint64_t valid, meas; uint32_t en[DPEMU_MAX_CORES], id[DPEMU_MAX_CORES];
                      uint32_t snap_ready; uint32_t snap_data[DPEMU_MAX_CORES]; };

rtl_fproc_tb *rtl_fproc_tb_new(uint32_t mode, uint32_t n, uint32_t lut_mask, const uint64_t *lut_table)
{
    rtl_fproc_tb *tb = (rtl_fproc_tb *)calloc(1, sizeof(rtl_fproc_tb));
    rtl_fproc_init(&tb->f, mode, n, lut_mask, lut_table);
    return tb;
}
void rtl_fproc_tb_free(rtl_fproc_tb *tb) { free(tb); }
void rtl_fproc_tb_set(rtl_fproc_tb *tb, int reset, uint64_t meas, uint64_t valid, uint64_t enable_mask,
                      const uint32_t *id)
{
    tb->reset = reset; tb->meas = meas; tb->valid = valid;
    for (uint32_t c = 0; c < tb->f.n; c++) { tb->en[c] = (uint32_t)((enable_mask >> c) & 1); if (id) tb->id[c] = id[c]; }
}
void rtl_fproc_tb_edge(rtl_fproc_tb *tb)
{
    rtl_fproc_eval(&tb->f, tb->valid, tb->meas);
    tb->snap_ready = 0;
    for (uint32_t c = 0; c < tb->f.n; c++) {
        if (tb->f.out_ready[c]) tb->snap_ready |= 1u << c;
        tb->snap_data[c] = tb->f.out_data[c];
    }
    rtl_fproc_commit(&tb->f, tb->reset, tb->valid, tb->meas, tb->en, tb->id);
}
uint32_t rtl_fproc_tb_ready(const rtl_fproc_tb *tb) { return tb->snap_ready; }
uint32_t rtl_fproc_tb_data(const rtl_fproc_tb *tb, int c) { return tb->snap_data[c]; }

/* ---------------------------------------------------------------------- */
/* batch driver with the dpemu output format (t = cycle - T0: first DECODE) */
/* ---------------------------------------------------------------------- */

static void put_event(oracle_lane_out *lo, uint32_t cap, uint32_t t, const rtl_core_comb *o, uint32_t kind)
{
    if (lo->n_events < cap) {
        uint32_t *e = lo->ev + 4 * lo->n_events;
        e[0] = t;
        e[1] = (o->env & 0xFFFFFF) | ((o->cfg & 0xF) << 24) | (kind << 28);
        e[2] = (o->phase & 0x1FFFF) | ((o->freq & 0x1FF) << 17);
        e[3] = o->amp & 0xFFFF;
    } else lo->flags |= DPEMU_F_EVENT_OVF;
    lo->n_events++;
}

static void put_trace(oracle_lane_out *lo, uint32_t cap, uint32_t t, uint32_t addr, uint32_t val)
{
    if (lo->n_trace < cap) {
        uint32_t *e = lo->tr + 4 * lo->n_trace;
        e[0] = t; e[1] = addr; e[2] = val; e[3] = 0;
    } else lo->flags |= DPEMU_F_TRACE_OVF;
    lo->n_trace++;
}

/*
 * Run one shot for `horizon` cycles past the first decode.  Per core, fills
 * `out[c]`: events, trace, measurements, t_end/qclk_end/ip of DONE, n_instr.
 * Returns 1 if every core reached DONE.
 */
int rtl_run_shot(const oracle_shot_cfg *cfg, const uint32_t *const *progs, const uint32_t *n_instr,
                 uint64_t shot, uint32_t horizon, uint32_t ev_cap, uint32_t tr_cap,
                 uint32_t meas_cap, oracle_lane_out *out)
{
    rtl_shot *s = (rtl_shot *)calloc(1, sizeof(rtl_shot));
    const uint32_t C = cfg->cores;
    uint32_t instr_addr[DPEMU_MAX_CORES] = {0}, last_qclk[DPEMU_MAX_CORES] = {0};
    for (uint32_t c = 0; c < C; c++) {
        out[c].n_events = out[c].n_trace = out[c].n_meas = out[c].n_instr = 0;
        out[c].flags = 0; out[c].status = 0; out[c].meas_bits = 0;
        out[c].t_end = out[c].ip = out[c].qclk_end = 0;
    }
    rtl_shot_init(s, cfg, progs, n_instr, shot);
    int all_done = 0;
    for (uint64_t cyc = 0; cyc <= (uint64_t)horizon + T0 + 2; cyc++) {
        uint32_t nm_before[DPEMU_MAX_CORES];
        for (uint32_t c = 0; c < C; c++) nm_before[c] = s->n_meas[c];
        rtl_shot_step(s, NULL);
        uint32_t t = (uint32_t)(cyc - T0);
        int done_now = 1;
        for (uint32_t c = 0; c < C; c++) {
            const rtl_core_comb *o = &s->core[c].comb;
            oracle_lane_out *lo = &out[c];
            if (o->load_en && lo->status == 0) { instr_addr[c] = o->load_addr; lo->n_instr++; }
            if (cyc >= T0) {
                if (o->cstrobe) put_event(lo, ev_cap, t, o, DPEMU_EV_STROBE);
                if (o->pulse_reset) put_event(lo, ev_cap, t, o, DPEMU_EV_PULSE_RESET);
                if (o->reg_we) put_trace(lo, tr_cap, t + 1, o->reg_wa, o->reg_wd);
                if (o->qclk_load) put_trace(lo, tr_cap, t + 1, DPEMU_TRACE_QCLK_LOAD, o->reg_wd + 3);
                if (o->qclk_rst_ctrl) put_trace(lo, tr_cap, t + 1, DPEMU_TRACE_QCLK_RST, 0);
                if (o->done_gate && lo->status == 0) {
                    lo->status = DPEMU_ST_DONE;
                    lo->t_end = t - 1;
                    lo->qclk_end = last_qclk[c];
                    lo->ip = instr_addr[c];
                }
            }
            if (s->n_meas[c] != nm_before[c]) {
                uint32_t m = s->n_meas[c] - 1;
                rtl_meas_q *q = &s->mq[c];
                uint32_t slot = (q->tail - 1) % RTL_MQ;
                if (m < meas_cap) {
                    lo->meas[2 * m] = (uint32_t)(q->t[slot] - T0);
                    lo->meas[2 * m + 1] = q->bit[slot];
                    if (lo->acc) { lo->acc[2 * m] = s->ro_acc[c][slot][0]; lo->acc[2 * m + 1] = s->ro_acc[c][slot][1]; }
                } else lo->flags |= DPEMU_F_MEAS_OVF;
                if (m < 32 && q->bit[slot]) lo->meas_bits |= 1u << m;
            }
            last_qclk[c] = o->qclk;
            if (!lo->status) done_now = 0;
        }
        if (done_now) { all_done = 1; break; }
    }
    for (uint32_t c = 0; c < C; c++) {
        out[c].n_meas = s->n_meas[c];
        memcpy(out[c].regs, s->core[c].regs, sizeof(out[c].regs));
    }
    free(s);
    return all_done;
}

/* ---------------------------------------------------------------------- */
/* per-clock batch: the CPU baseline closest to the Verilator testbench     */
/* ---------------------------------------------------------------------- */
/*
 * Shots [shot_begin, shot_begin + n_shots) of a dpemu program set, one
 * rtl_run_shot per shot, OpenMP over shots: the per-clock analogue of the
 * reference's Verilator/cocotb run (cocotb/proc/Makefile:1-14), which cannot
 * run in this image.  Events, traces and measurements go to per-thread
 * buffers of the config's caps (the same work as a dpemu run); the summary
 * rows (dpemu layout, include/dpemu.h) go to `summary` when it is non-null.
 * `horizon`: cycles simulated past the first decode at most.  ro_words /
 * ro_hdr: the DEMOD frequency tables, as fast_run takes them (or NULL).  Returns the
 * number of shots whose every core reached DONE, or -1 for a bad config or
 * a failed scratch allocation (C x event_cap x 16 B per thread).
 */
int64_t rtl_run_batch(const dpemu_config *cfg, const uint32_t *words, const uint32_t *offsets,
                      const uint32_t *n_instr, const uint32_t *prog_table, uint64_t shot_begin,
                      uint64_t n_shots, uint32_t horizon, uint32_t *summary, int n_threads,
                      const uint32_t *ro_words, const uint32_t *ro_hdr)
{
    const uint32_t C = cfg->cores_per_shot;
    if (C == 0 || C > DPEMU_MAX_CORES || (C & (C - 1))) return -1;
    oracle_shot_cfg sc;
    memset(&sc, 0, sizeof sc);
    sc.cores = C; sc.fproc_mode = cfg->fproc_mode; sc.sync_external = 0;
    sc.meas_elem = cfg->meas_elem; sc.meas_latency = cfg->meas_latency; sc.sync_latency = cfg->sync_latency;
    sc.sync_mask = cfg->sync_mask; sc.seed = cfg->seed; sc.lut_mask = cfg->lut_mask;
    memcpy(sc.p1_threshold, cfg->p1_threshold, sizeof sc.p1_threshold);
    memcpy(sc.lut_table, cfg->lut_table, sizeof sc.lut_table);
    sc.meas_model = cfg->meas_model; sc.ro_sep = cfg->ro_sep; sc.ro_sigma = cfg->ro_sigma;
    sc.ro_thr = cfg->ro_thr; sc.ro_win = cfg->ro_win;
    sc.ro = *cfg;
    const uint32_t ev_cap = cfg->event_cap ? cfg->event_cap : 1, tr_cap = cfg->trace_cap ? cfg->trace_cap : 1;
    const uint32_t ms_cap = cfg->meas_cap ? cfg->meas_cap : 1;
    int64_t done = 0;
    int oom = 0;                 /* any thread's scratch allocation failed */
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    #pragma omp parallel reduction(+ : done) reduction(| : oom)
    {
        oracle_lane_out *lo = (oracle_lane_out *)calloc(C, sizeof(oracle_lane_out));
        uint32_t *ev = (uint32_t *)malloc((size_t)C * ev_cap * 16);
        uint32_t *tr = (uint32_t *)malloc((size_t)C * tr_cap * 16);
        uint32_t *ms = (uint32_t *)malloc((size_t)C * ms_cap * 8);
        const int bad = !lo || !ev || !tr || !ms;
        oom |= bad;
        for (uint32_t c = 0; c < C && !bad; c++) {
            lo[c].ev = ev + (size_t)c * ev_cap * 4;
            lo[c].tr = tr + (size_t)c * tr_cap * 4; lo[c].meas = ms + (size_t)c * ms_cap * 2;
        }
        const uint32_t *progs[DPEMU_MAX_CORES];
        uint32_t ni[DPEMU_MAX_CORES];
        oracle_shot_cfg *tc = (oracle_shot_cfg *)malloc(sizeof sc);   /* this thread's copy (DEMOD tables) */
        if (tc) *tc = sc;
        else oom = 1;
        #pragma omp for schedule(dynamic, 4)
        for (int64_t si = 0; si < (int64_t)n_shots; si++) {
            if (bad || !tc) continue;   /* (no break inside an omp for) */
            const uint64_t shot = shot_begin + (uint64_t)si;
            const uint32_t g = (uint32_t)((shot / cfg->shots_per_group) % cfg->n_groups);
            for (uint32_t c = 0; c < C; c++) {
                const uint32_t p = prog_table[(uint64_t)g * C + c];
                progs[c] = words + 4 * (uint64_t)offsets[p];
                ni[c] = n_instr[p];
                if (ro_words && ro_hdr) {
                    const uint32_t *h = ro_hdr + 4 * (uint64_t)p;
                    tc->ro_tab[c][0] = ro_words + h[0]; tc->ro_len[c][0] = h[1];
                    tc->ro_tab[c][1] = ro_words + h[2]; tc->ro_len[c][1] = h[3];
                }
            }
            done += rtl_run_shot(tc, progs, ni, shot, horizon, cfg->event_cap, cfg->trace_cap, cfg->meas_cap, lo);
            if (summary)
                for (uint32_t c = 0; c < C; c++) {
                    const uint64_t L = cfg->lane_order == DPEMU_LANES_SHOT_MAJOR ? (uint64_t)si * C + c
                                                                                 : (uint64_t)c * n_shots + (uint64_t)si;
                    uint32_t *sm = summary + 8 * L;                          /* include/dpemu.h lane order */
                    sm[0] = lo[c].t_end;
                    sm[1] = (lo[c].ip & 0xFFFF) | ((lo[c].status & 0xFF) << 16) | ((lo[c].flags & 0xFF) << 24);
                    sm[2] = lo[c].n_events; sm[3] = lo[c].n_instr; sm[4] = lo[c].qclk_end;
                    sm[5] = lo[c].n_meas; sm[6] = lo[c].meas_bits; sm[7] = lo[c].n_trace;
                }
        }
        free(lo); free(ev); free(tr); free(ms); free(tc);
    }
    return oom ? -1 : done;
}
