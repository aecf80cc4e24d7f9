/*
 * oracle/oracle.h -- TEST INFRASTRUCTURE: CPU restatements used as checkers.
 *
 *   oracle_rtl  (rtl_model.c)  literal per-clock restatement of the hdl/ modules
 *   oracle_fast (fast_model.c) event-driven restatement: the closed-form
 *               decode-to-decode timing of SURVEY.md §2.4, pinned to
 *               oracle_rtl by fuzzing (tests/test_fast_vs_rtl.py)
 *   oracle_dds  (dds_ref.c)    fixed-point DDS restatement
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline.
 */
#ifndef DPEMU_ORACLE_H
#define DPEMU_ORACLE_H

#include <stdint.h>
#include "../include/dpemu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_FPROC_EXTERNAL 99   /* testbench drives fproc_ready/data (cocotb style) */

uint32_t oracle_alu(uint32_t ctrl, uint32_t in0, uint32_t in1);
void oracle_pulse_reg(uint32_t pr[5], const uint32_t lc[4], uint32_t reg_in, int write_en);
uint32_t oracle_philox_u32(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m);
void oracle_philox4(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m, uint32_t out[4]);
/* outcome of measurement m of (shot, core): the prepared state drawn against
 * thr, or (meas_model READOUT) the discriminated readout of a pulse with amp
 * word `amp` (include/dpemu.h, dpemu_config) */
uint32_t oracle_meas_bit(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m, uint32_t thr, uint32_t amp,
                         uint32_t meas_model, int32_t ro_sep, uint32_t ro_sigma, int32_t ro_thr,
                         uint32_t ro_win, uint32_t env);

/* ---- readout demodulation model (readout.c; meas_model DPEMU_MEAS_DEMOD) ---- */
typedef struct {
    uint32_t have;             /* a readout-drive strobe was seen                   */
    uint32_t t, env, pp, amp;  /* its cycle, env word, phase | freq << 17, amp word */
} oracle_ro_drive;
int64_t oracle_sin33(int64_t x);                      /* sin(2 pi x / 2^33) * 2^61 */
int64_t oracle_dirichlet_q16(uint32_t n, uint32_t beta);
uint32_t oracle_ro_words(uint32_t env);               /* env length field, 0 (CW) = 4096 */
uint32_t oracle_ro_freq(const uint32_t *tab, uint32_t len, uint32_t pp);
/* meas_valid of a readout at t_lo after one valid at last_tv (0: none) */
uint32_t oracle_demod_valid(const dpemu_config *cfg, uint32_t t_lo, uint32_t env_lo, uint32_t last_tv);
/* outcome of measurement m; acc = the accumulated {I, Q} */
uint32_t oracle_demod(const dpemu_config *cfg, uint64_t shot, uint32_t core, uint32_t m, uint32_t t_lo,
                      uint32_t env_lo, uint32_t pp_lo, uint32_t f_lo, const oracle_ro_drive *d, uint32_t f_d,
                      uint32_t t_ref, int32_t acc[2]);

/* ---- per-clock model ---------------------------------------------------- */
typedef struct {
    uint8_t reset_reg, reset_sr, qclk_trig, cstrobe_p;
    uint8_t state; uint32_t mwc;
    uint32_t lc[4];
    uint32_t ipv, ipv_inc, ra[3];
    uint32_t alu_in0, alu_in1, alu_out, qclk;
    uint32_t p_env, p_phase, p_freq, p_amp, p_cfg; uint8_t p_cstrobe;
    uint8_t reg_we; uint32_t reg_wa, reg_wd;
} rtl_core_regs;

typedef struct {
    uint32_t state, opcode, qclk;
    uint32_t cstrobe, env, phase, freq, amp, cfg;      /* pulse_iface */
    uint32_t pulse_reset, done_gate, sync_enable, fproc_enable, fproc_id;
    uint32_t instr_ptr, load_en, load_addr;
    uint32_t cmd_buf_out[4];
    uint32_t reg_we, reg_wa, reg_wd, qclk_load, qclk_rst_ctrl;
} rtl_core_comb;

typedef struct {
    /* registers (proc.sv, ctrl.v, instr_ptr.v, cmd_mem.v, alu.v, qclk.v, pulse_reg.sv) */
    uint8_t reset_reg, reset_sr, qclk_trig, cstrobe_p;
    uint8_t state; uint32_t mwc;
    uint32_t lc[4];
    uint32_t ipv, ipv_inc, ra[3];
    uint32_t regs[16];
    uint32_t alu_in0, alu_in1, alu_out, qclk;
    uint32_t p_env, p_phase, p_freq, p_amp, p_cfg; uint8_t p_cstrobe;
    /* program */
    const uint32_t *prog; uint32_t n_instr, addr_mask;
    /* this clock */
    rtl_core_comb comb;
    rtl_core_regs nxt;
} rtl_core;

void rtl_core_init(rtl_core *c, const uint32_t *prog, uint32_t n_instr, int addr_width);
void rtl_core_eval(rtl_core *c, int reset, int fproc_ready, uint32_t fproc_data, int sync_ready);
void rtl_core_commit(rtl_core *c);

typedef struct {
    uint32_t cores;          /* C */
    uint32_t fproc_mode;     /* DPEMU_FPROC_MEAS / _LUT / ORACLE_FPROC_EXTERNAL */
    uint32_t sync_external;  /* testbench drives sync_ready */
    uint32_t meas_elem, meas_latency, sync_latency;
    uint64_t sync_mask, seed;
    uint32_t lut_mask;
    uint32_t p1_threshold[DPEMU_MAX_CORES];
    uint64_t lut_table[256];
    uint32_t meas_model;
    int32_t ro_sep;
    uint32_t ro_sigma;
    int32_t ro_thr;
    uint32_t ro_win;
    /* DEMOD: the run's config (its seed, thresholds and ro_* fields are the ones
     * read) and each core's drive / LO frequency tables */
    dpemu_config ro;
    const uint32_t *ro_tab[DPEMU_MAX_CORES][2];
    uint32_t ro_len[DPEMU_MAX_CORES][2];
} oracle_shot_cfg;

#define RTL_MQ 64
typedef struct { uint64_t t[RTL_MQ]; uint8_t bit[RTL_MQ]; uint32_t head, tail; } rtl_meas_q;

typedef struct {
    int reset;
    int drive_meas; uint64_t meas_valid, meas;
    int fproc_ready[DPEMU_MAX_CORES]; uint32_t fproc_data[DPEMU_MAX_CORES];
    int sync_ready;
} rtl_ext_inputs;

/* fproc back end: fproc_meas.sv, or core_state_mgr.sv + meas_lut.sv */
typedef struct {
    uint32_t mode, n, addr_mask, lut_mask;
    uint64_t lut_table[256];
    /* fproc_meas registers */
    uint8_t arm[DPEMU_MAX_CORES], ready[DPEMU_MAX_CORES];
    uint32_t addr[DPEMU_MAX_CORES], data[DPEMU_MAX_CORES];
    uint64_t meas_reg;
    /* core_state_mgr / meas_lut registers */
    uint8_t cs[DPEMU_MAX_CORES];
    uint8_t lut_state; uint64_t lut_valid, lut_addr;
    /* this clock */
    int out_ready[DPEMU_MAX_CORES]; uint32_t out_data[DPEMU_MAX_CORES];
    int lut_ready; uint64_t lut_v, lut_a;
} rtl_fproc;

void rtl_fproc_init(rtl_fproc *f, uint32_t mode, uint32_t n, uint32_t lut_mask, const uint64_t *lut_table);
void rtl_fproc_eval(rtl_fproc *f, uint64_t valid, uint64_t meas);
void rtl_fproc_commit(rtl_fproc *f, int reset, uint64_t valid, uint64_t meas,
                      const uint32_t *enable, const uint32_t *id);

typedef struct {
    oracle_shot_cfg cfg;
    uint64_t shot, cycle;
    rtl_core core[DPEMU_MAX_CORES];
    rtl_fproc fp;
    uint64_t sync_mask;
    /* measurement model */
    rtl_meas_q mq[DPEMU_MAX_CORES];
    uint32_t n_meas[DPEMU_MAX_CORES];
    uint64_t cur_valid, cur_meas;
    /* DEMOD: each core's latest readout-drive strobe and pulse_reset (dpemu
     * times, cycle - T0), its last meas_valid cycle and accumulated {I, Q} */
    oracle_ro_drive ro_d[DPEMU_MAX_CORES];
    uint32_t ro_tref[DPEMU_MAX_CORES];
    uint64_t ro_last_tv[DPEMU_MAX_CORES];
    int32_t ro_acc[DPEMU_MAX_CORES][RTL_MQ][2];
    /* sync controller */
    uint64_t sync_arrived; int sync_pend; uint64_t sync_t;
} rtl_shot;

typedef struct rtl_tb rtl_tb;
rtl_tb *rtl_tb_new(void);
void rtl_tb_free(rtl_tb *tb);
void rtl_tb_set(rtl_tb *tb, int reset, int fproc_ready, uint32_t fproc_data, int sync_ready);
void rtl_tb_write(rtl_tb *tb, int en, uint32_t addr, const uint32_t *word);
void rtl_tb_edge(rtl_tb *tb);
const rtl_core_comb *rtl_tb_snap(const rtl_tb *tb);
uint32_t rtl_tb_reg(const rtl_tb *tb, int i);

typedef struct rtl_fproc_tb rtl_fproc_tb;
rtl_fproc_tb *rtl_fproc_tb_new(uint32_t mode, uint32_t n, uint32_t lut_mask, const uint64_t *lut_table);
void rtl_fproc_tb_free(rtl_fproc_tb *tb);
void rtl_fproc_tb_set(rtl_fproc_tb *tb, int reset, uint64_t meas, uint64_t valid, uint64_t enable_mask,
                      const uint32_t *id);
void rtl_fproc_tb_edge(rtl_fproc_tb *tb);
uint32_t rtl_fproc_tb_ready(const rtl_fproc_tb *tb);
uint32_t rtl_fproc_tb_data(const rtl_fproc_tb *tb, int c);

void rtl_shot_init(rtl_shot *s, const oracle_shot_cfg *cfg, const uint32_t *const *progs,
                   const uint32_t *n_instr, uint64_t shot_index);
void rtl_shot_step(rtl_shot *s, const rtl_ext_inputs *ext);

/* per-lane result of one shot, dpemu formats */
typedef struct {
    uint32_t status, flags, t_end, ip, qclk_end, n_instr;
    uint32_t n_events, n_trace, n_meas, meas_bits;
    uint32_t regs[16];
    uint32_t *ev;      /* [ev_cap][4] event records (include/dpemu.h) */
    uint32_t *tr;      /* [tr_cap][4] */
    uint32_t *meas;    /* [meas_cap][2] */
    int32_t *acc;      /* [meas_cap][2] accumulated {I, Q} (DEMOD), or NULL */
} oracle_lane_out;

int rtl_run_shot(const oracle_shot_cfg *cfg, const uint32_t *const *progs, const uint32_t *n_instr,
                 uint64_t shot, uint32_t horizon, uint32_t ev_cap, uint32_t tr_cap,
                 uint32_t meas_cap, oracle_lane_out *out);

/* per-clock batch over shots (OpenMP), dpemu summary rows; returns shots all-DONE */
int64_t rtl_run_batch(const dpemu_config *cfg, const uint32_t *words, const uint32_t *offsets,
                      const uint32_t *n_instr, const uint32_t *prog_table, uint64_t shot_begin,
                      uint64_t n_shots, uint32_t horizon, uint32_t *summary, int n_threads,
                      const uint32_t *ro_words, const uint32_t *ro_hdr);

/* ---- event-driven model, dpemu_run-compatible batch entry ------------------ */
/* ro_words / ro_hdr: the DEMOD frequency tables (dpemu_load_readout_freqs), ro_hdr
 * [n_programs][4] = drv_off, drv_len, lo_off, lo_len; NULL when not DEMOD */
int fast_run(const dpemu_config *cfg, const uint32_t *words, const uint32_t *offsets,
             const uint32_t *n_instr, const uint32_t *prog_table, uint64_t shot_begin,
             uint64_t n_shots, const dpemu_outputs *out, int n_threads,
             const uint32_t *ro_words, const uint32_t *ro_hdr);

/* ---- DDS restatement --------------------------------------------------------- */
void oracle_dds_sin_lut(int16_t *out4096);
typedef struct {
    uint32_t n_channels, n_lanes, n_samples, event_cap;
    const uint32_t *ch;          /* [n_channels][8]: lane, elem, spc, interp, env_off, env_len, freq_off, freq_len */
    const uint32_t *summary;     /* [n_lanes][8] */
    const uint32_t *events;      /* [event_cap][n_lanes][4] */
    const uint32_t *env, *freq;
    uint32_t *iq;                /* [n_channels][n_samples] */
} oracle_dds_args;
void oracle_dds(const oracle_dds_args *a, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
