/*
 * dpemu.h -- C ABI of the MI355X-native batched QubiC distributed-processor
 * emulator (libdpemu.so).
 *
 * The emulator executes the 128-bit machine code that distproc's assembler
 * writes into cmd_mem (python/distproc/assembler.py:341-429,623-641) across
 * many (shot, core) lanes, cycle-exact against the gateware:
 *   proc core           hdl/proc.sv:9-171, ctrl.v:55-595, alu.v, instr_ptr.v,
 *                       qclk.v, reg_file.v, cmd_mem.v (READ_LATENCY=3)
 *   pulse emission      hdl/pulse_reg.sv:16-107, pulse_iface.sv
 *   measurement fproc   hdl/fproc_meas.sv, fproc_lut.sv, core_state_mgr.sv,
 *                       meas_lut.sv
 *   sync barrier        hdl/sync_iface.sv + ctrl.v:347-363,510-552 (the
 *                       controller itself is build-defined)
 * and synthesises DDS I/Q samples from the pulse events (build-defined DDS).
 *
 * Each entry point replaces one piece of the reference simulation path
 * (SURVEY.md §8b): the cocotb/Verilator harness of toplevel_sim
 * (sim_modules/toplevel_sim.sv:13-33; cocotb/proc/test_proc.py:29-38 loads
 * cmd_mem, drives reset/fproc/sync, samples pulse_iface every clock).
 *
 * Conventions: return 0 on success, a negative DPEMU_E* code on failure (no
 * exceptions cross the ABI; dpemu_last_error() has the message).  Caller
 * owns every pointer it passes.  Device-pointer outputs must be device
 * memory of the context's device; NULL skips that output.  A context is not
 * re-entrant (one host thread at a time); use one per device (one process
 * per GPU).  Work a context enqueues runs in call order even across streams:
 * a call on a stream other than the previous call's first makes that stream
 * wait for the previous call's work (the context's scratch buffers and
 * uploaded constants are shared by its calls).
 */
#ifndef DPEMU_H
#define DPEMU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPEMU_ABI_VERSION 8

/* ---- error codes ---------------------------------------------------- */
#define DPEMU_OK            0
#define DPEMU_E_INVALID   (-22)   /* bad argument / inconsistent config  */
#define DPEMU_E_NOMEM     (-12)   /* device allocation failed            */
#define DPEMU_E_DEVICE     (-5)   /* HIP runtime error                   */
#define DPEMU_E_NOPROG     (-2)   /* run before load_programs            */

/* ---- lane terminal status (summary.w1 bits 23:16) -------------------- */
#define DPEMU_ST_DONE        1    /* decoded DONE (1010) or opcode 0000 (ctrl.v:365-397) */
#define DPEMU_ST_MAX_CYCLES  2    /* next decode, or a wait's end, beyond max_cycles     */
#define DPEMU_ST_HUNG_OPCODE 3    /* opcode[7:4] in 1101..1111: DECODE forever (ctrl.v:399-414) */
#define DPEMU_ST_DEADLOCK    4    /* sync / fproc wait that can never complete           */

/* ---- lane flags (summary.w1 bits 31:24) ------------------------------ */
#define DPEMU_F_LATE          0x01 /* trig/idle decoded after cmd_time: waits for qclk wrap */
#define DPEMU_F_EVENT_OVF     0x02 /* more events than event_cap (count still exact)        */
#define DPEMU_F_TRACE_OVF     0x04 /* more register-trace records than trace_cap            */
#define DPEMU_F_MEAS_OVF      0x08 /* more measurements than meas_cap                       */
#define DPEMU_F_DOUBLE_STROBE 0x10 /* trig at the first decode with cmd_time 0: the reset
                                      hold keeps qclk at 0 two cycles -> two cstrobes      */
#define DPEMU_F_GUARD         0x20 /* internal error: interpreter iteration guard tripped    */

/* ---- fproc back ends --------------------------------------------------*/
#define DPEMU_FPROC_MEAS 0        /* hdl/fproc_meas.sv: latest stored bit, ready at D+2   */
#define DPEMU_FPROC_LUT  1        /* hdl/fproc_lut.sv: id==0 wait own meas, else LUT      */

/* ---- event kinds (event.w2 bits 31:28) ------------------------------- */
#define DPEMU_EV_STROBE      0    /* pulse_iface.cstrobe high: pulse register snapshot    */
#define DPEMU_EV_PULSE_RESET 1    /* pulse_iface.reset high (PULSE_RESET decode cycle)    */

/* ---- register-trace pseudo addresses ---------------------------------- */
#define DPEMU_TRACE_QCLK_LOAD 16  /* INC_QCLK loaded qclk (value = qclk at t)             */
#define DPEMU_TRACE_QCLK_RST  17  /* SYNC reset qclk (value 0 at t)                       */

/* execution knobs (dpemu_config.exec_flags): results never depend on them; the
 * parity tests run every variant against the oracle */
#define DPEMU_X_PROG_LDS    0x1   /* run non-pulse-only programs on the general interpreter with each
                                     workgroup's programs staged in LDS when they fit */
#define DPEMU_X_HIST_DIRECT 0x4   /* outcome histogram: atomics straight into out->hist       */
#define DPEMU_X_HIST_REPL   0x8   /* outcome histogram: privatised replicas + reduce          */
#define DPEMU_X_PROG_MAJOR  0x10  /* fetch from the program-major image, not the command-major copy */
#define DPEMU_X_GENERAL     0x20  /* run every program on the general interpreter (interp_kernel) */
#define DPEMU_X_MACRO_DIRECT 0x40 /* branch-free register programs: per-lane macro fetch (macro_kernel),
                                     not the LDS-staged program chunks (macro_staged_kernel) */
#define DPEMU_X_STREAM_EVENTS 0x80 /* cache hint: branch-free register programs store their event rows
                                     nontemporal (whole-wave stores; others write-back).  Workload-
                                     dependent: config 4 two-qubit RB -9 %, RB-shaped programs +10 %
                                     (profiles/r06_stpol_ab.json) */

#define DPEMU_MAX_CORES 64
#define DPEMU_MEAS_LOOKUP 16      /* a core's first 16 measurements are visible to fproc;
                                     later ones set DPEMU_F_MEAS_OVF and are invisible  */
#define DPEMU_LUT_FIRE_CAP 16     /* meas_lut fires recorded per shot (later fires lost) */

/*
 * Timebase: cycle t = 0 is the first DECODE after reset.  qclk(0) = qclk(1) = 0
 * (reset hold, proc.sv:125-136), qclk(t) = t - 1 afterwards until INC_QCLK or
 * SYNC reload it.  All times are emulated fabric clocks (2 ns at 500 MHz).
 */
typedef struct dpemu_config {
    uint32_t cores_per_shot;   /* C: power of two, 1..64; lane = shot*C + core        */
    uint32_t n_groups;         /* program groups; group(s) = (s/shots_per_group)%n_groups */
    uint32_t shots_per_group;  /* >= 1                                                  */
    uint32_t max_cycles;       /* <= 2^31 - 64                                          */
    uint32_t event_cap;        /* event slots per lane (<= DPEMU_MAX_EVENT_CAP)           */
    uint32_t trace_cap;        /* register-trace slots per lane (0 = no trace; <= DPEMU_MAX_EVENT_CAP) */
    uint32_t meas_cap;         /* measurement slots per lane (<= 32)                     */
    uint32_t fproc_mode;       /* DPEMU_FPROC_*                                          */
    uint32_t meas_elem;        /* strobe with (cfg & 3) == meas_elem is a readout; 0xFF none */
    uint32_t meas_latency;     /* readout strobe -> meas_valid, clocks (>= 1)           */
    uint32_t sync_latency;     /* last sync enable -> sync.ready, clocks (>= 1)         */
    uint32_t exec_flags;       /* DPEMU_X_* execution knobs (results never depend on them) */
    uint64_t sync_mask;        /* participant cores (bit c); 0 = all C cores             */
    uint64_t seed;             /* Philox4x32-10 key                                      */
    uint32_t lut_mask;         /* meas_lut mask (nonzero), meas_lut.sv:16                */
    uint32_t meas_model;       /* DPEMU_MEAS_STATE: outcome = prepared state; DPEMU_MEAS_READOUT:
                                  the discriminated readout signal (ro_* below)            */
    uint32_t p1_threshold[DPEMU_MAX_CORES]; /* P(state=1) = thr/2^32; 0xFFFFFFFF = always 1 */
    uint64_t lut_table[256];   /* meas_lut table: lut_out = table[addr], bit c -> core c */
    /* readout model (meas_model = DPEMU_MEAS_READOUT), per readout strobe with amp word A:
     *   z = Irwin-Hall(4) of the 16-bit halves of Philox words 1, 2, minus 131070
     *   x = (state ? +1 : -1) * ((ro_sep * A) >> 16) + ((z * ro_sigma) >> 16)   (int64)
     *   outcome = x > ro_thr
     * with ro_win != 0 the separation also scales with the readout window:
     *   s = (s * (min(W, ro_win) * floor(2^24 / ro_win))) >> 24   (int64)
     * unless W == 0: a CW envelope word (length field 0) plays until the next
     * pulse, so it integrates the whole window and s is not scaled
     * W = the strobe's envelope-length field (env word bits 23:12, in env words)
     * -- a window shorter than ro_win integrates less signal                  */
    int32_t  ro_sep;           /* half the state separation at full readout amplitude    */
    uint32_t ro_sigma;         /* noise scale, Q16 (noise sigma = ro_sigma / 2^16 * 37837.6) */
    int32_t  ro_thr;           /* discriminator threshold                                */
    uint32_t ro_win;           /* reference readout window (env words, < 4096); 0 = amplitude only */
    uint32_t hist_assign;      /* 0: out->hist += this run's counts; 1: out->hist = this run's
                                  counts (no separate zeroing launch before each run)        */
    uint32_t lane_order;       /* DPEMU_LANES_CORE_MAJOR (0) or DPEMU_LANES_SHOT_MAJOR (1), below */
    /* readout demodulation model (meas_model = DPEMU_MEAS_DEMOD, ABI 8).
     * The return of the lane's latest readout-drive strobe (cfg & 3 == ro_drv_elem,
     * t_d <= t_lo) is mixed with the readout strobe's own LO (cfg & 3 == meas_elem,
     * at t_lo) and accumulated per clock over their overlap; both phases follow the
     * DDS phase accumulator, F * (k - t_ref) + phase17 << 15 (t_ref = the latest
     * pulse_reset <= t_lo; F = the 32-bit frequency word of the pulse's freq index,
     * dpemu_load_readout_freqs).  Per clock k of the overlap, with s the prepared state:
     *   return  amp_d * ro_gain[s] / 2^16 at phase F_d (k - ro_delay - t_ref)
     *           + phase_d << 15 + ro_theta[s]
     *   acc    += return * conj(LO)   (int32 I / Q, closed form: exact integer
     *                                   arithmetic of DESIGN.md §2, oracle/readout.c)
     *   acc    += noise: (z_I, z_Q) * ro_sigma / 2^16 (Hadamard pairs of 4 Philox halves)
     *   x       = (acc_I * axis_I + acc_Q * axis_Q) >> 15, axis = ro_axis[core]
     *   outcome = x > ro_thr, meas_valid at max(t_lo + window + meas_latency,
     *             the lane's previous meas_valid + 1)   (an in-order readout pipeline)
     * window = the readout strobe's env length field (bits 23:12) * ro_cpw clocks
     * (length 0: a CW envelope, 4096 words); the drive pulse lasts likewise.       */
    uint32_t ro_drv_elem;      /* element of the readout drive (rdrv) strobes, 0..3, != meas_elem */
    uint32_t ro_cpw;           /* clocks per env word of the rdrv / rdlo pulses, 1..8 (4 for
                                  channel_config.json's rdrv 16 samples/clk interp 16, rdlo 4 / 4) */
    uint32_t ro_delay;         /* drive -> ADC return delay, clocks (< 2^20)                */
    uint32_t ro_theta[2];      /* return phase shift for prepared state 0 / 1 (2^32 = 2 pi)  */
    uint32_t ro_gain[2];       /* return amplitude for state 0 / 1, Q16 (<= 65536)         */
    uint32_t ro_axis[DPEMU_MAX_CORES]; /* discriminator axis per core, Q15: I16 low | Q16 high */
} dpemu_config;

#define DPEMU_MEAS_STATE   0
#define DPEMU_MEAS_READOUT 1
#define DPEMU_MEAS_DEMOD   2      /* rdlo demodulation of the rdrv return (ro_drv_elem ...) */
#define DPEMU_RO_CPW_MAX   8      /* ro_cpw bound: an accumulation window is <= 2^15 clocks   */

/* lane order of every per-lane output (dpemu_config.lane_order) */
#define DPEMU_LANES_CORE_MAJOR 0  /* lane = core * n_shots + (shot - shot_begin)                  */
#define DPEMU_LANES_SHOT_MAJOR 1  /* lane = (shot - shot_begin) * C + core: a shot's cores adjacent */

#define DPEMU_MAX_EVENT_CAP (1u << 20)   /* event / trace slots per lane (validate)  */

/*
 * Lanes: lane L = core * n_shots + (shot - shot_begin) -- core-major, so the
 * lanes of one core's shots are adjacent (the lanes that run one program in
 * lockstep write whole cache lines) -- or, with lane_order SHOT_MAJOR,
 * L = (shot - shot_begin) * C + core (a shot's cores adjacent: the layout the
 * fproc / sync interpreter writes as whole lines, since a wave holds whole
 * shots).
 *
 * Per-lane summary, 8 x u32:
 *   w0 t_end      decode cycle of DONE (done_gate from t_end+1) or of the stop
 *   w1 ip[15:0] | status[23:16] | flags[31:24]
 *   w2 n_events   strobe + pulse_reset events (may exceed event_cap)
 *   w3 n_instr    instructions decoded (DONE included)
 *   w4 qclk_end   qclk at t_end
 *   w5 n_meas     measurements taken
 *   w6 meas_bits  outcome of measurement m in bit m (m < 32)
 *   w7 n_trace    register-trace records (may exceed trace_cap)
 *
 * Event (slot-major: slot k of lane L at index k*n_lanes + L), one 16-B record
 * per pulse_iface strobe (hdl/pulse_iface.sv:2-6) or pulse reset:
 *   uint4 {t, env[23:0] | cfg<<24 | kind<<28, phase[16:0] | freq<<17, amp[15:0]}
 * (qclk at an event follows from t and the lane's qclk loads / resets, which
 * the register trace records)
 * Trace (slot-major): uint4 {t (first cycle the value is visible), addr, value, 0}
 * Meas  (slot-major): uint2 {valid cycle, bit}
 * Histogram: uint64 [n_groups][2^C] (C <= 12), key bit c = last outcome of core c.
 */
typedef struct dpemu_outputs {
    uint32_t *summary;    /* [n_lanes][8]                      */
    uint32_t *events;     /* [event_cap][n_lanes][4]           */
    uint32_t *trace;      /* [trace_cap][n_lanes][4]           */
    uint32_t *meas;       /* [meas_cap][n_lanes][2]            */
    uint32_t *regs;       /* [16][n_lanes] final register file */
    uint64_t *hist;       /* [n_groups][2^C], accumulated (or assigned: hist_assign) */
    uint64_t *hist_next;  /* optional, dpemu_run only: a second [n_groups][2^C] buffer, disjoint
                             from hist, that this run sets to zero in passing -- the buffer the
                             caller's next run accumulates into, so a pipeline of runs rotating
                             over three histogram buffers needs no zeroing launch (ABI 7) */
    int32_t  *acc;        /* [meas_cap][n_lanes][2] accumulated {I, Q} of each readout (the
                             accbuf of hwconfig.py:128,138-140); DEMOD runs only (ABI 8) */
} dpemu_outputs;

typedef struct dpemu_ctx dpemu_ctx;

/* Library / device --------------------------------------------------- */
int         dpemu_abi_version(void);
/* sizeof(dpemu_config), sizeof(dpemu_outputs), sizeof(dpemu_dds_channels) as
 * this library was compiled: a binding compares them with its own layout
 * before the first call (the version number alone does not catch a build
 * from a half-edited header).  out: 3 entries. */
int         dpemu_struct_sizes(uint64_t *out);
int         dpemu_create(int device, dpemu_ctx **out);
int         dpemu_destroy(dpemu_ctx *ctx);
const char *dpemu_last_error(dpemu_ctx *ctx);

/*
 * Programs: n_programs cmd_mem images.  `words` holds n_cmds little-endian
 * u128 commands as u32 quads (word i of the u128 = bits [32i+31:32i],
 * cmd_mem_iface.sv:19-21), i.e. 4 * n_cmds u32 words; program p starts at
 * COMMAND offsets[p] with n_instr[p] commands (assembler cmd_buf bytes
 * reinterpret directly).  n_cmds, offsets and n_instr all count 16-byte
 * commands; offsets[p] + n_instr[p] <= n_cmds for every p, else
 * DPEMU_E_INVALID (nothing past the caller's 16 * n_cmds bytes is read).  Fetch beyond
 * n_instr reads 0 (= DONE), as the zero-initialised 2^16-deep cmd_mem of
 * toplevel_sim does.  prog_table[g*C + c] = program run by core c of shots
 * in group g.  Replaces load_commands (cocotb/proc/test_proc.py:29-38).
 */
int dpemu_load_programs(dpemu_ctx *ctx, const uint32_t *words, uint64_t n_cmds, const uint32_t *offsets,
                        const uint32_t *n_instr, uint32_t n_programs,
                        const uint32_t *prog_table, uint32_t n_groups, uint32_t cores_per_shot);

/*
 * Frequency words of the DEMOD readout model (ABI 8), per loaded program p:
 * the readout drive element's freq index i reads words[drv_off[p] + i] when
 * i < drv_len[p], else 0; the LO element's reads words[lo_off[p] + i] (i <
 * lo_len[p]).  Each word is entry i's first word of the element's
 * freq_buffer, f / f_clk * 2^32 (python/distproc/asmparse.py:64-86; the
 * assembler's freq_buffers, assembler.py:510-516).  Arrays hold n_programs
 * entries (the count of the last dpemu_load_programs); offsets + lengths
 * must stay within n_words.  dpemu_load_programs clears the tables, and a
 * DEMOD run without them is DPEMU_E_INVALID.
 */
int dpemu_load_readout_freqs(dpemu_ctx *ctx, const uint32_t *words, uint64_t n_words, const uint32_t *drv_off,
                             const uint32_t *drv_len, const uint32_t *lo_off, const uint32_t *lo_len);

/* Emulate shots [shot_begin, shot_begin + n_shots) on `stream` (hipStream_t or
 * NULL).  n_lanes = n_shots * C.  Outputs are device pointers.  out->hist_next,
 * when set, is zeroed even for n_shots = 0; overlapping out->hist is
 * DPEMU_E_INVALID. */
int dpemu_run(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t shot_begin, uint64_t n_shots,
              const dpemu_outputs *out, void *stream);

/* Same, with host output pointers (the library stages device buffers);
 * host_out->hist_next must be NULL (DPEMU_E_INVALID otherwise). */
int dpemu_run_host(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t shot_begin,
                   uint64_t n_shots, const dpemu_outputs *host_out);

/*
 * DDS synthesis (build-defined fixed point; CPU restatement
 * oracle/dds_ref.c).  One channel = one (lane, element) pair: it plays the
 * lane's strobes whose cfg & 3 == element, with the lane's pulse_resets as
 * phase references, from the events dpemu_run wrote (slot-major, n_lanes
 * stride, count = min(summary n_events, event_cap)).  Env / freq tables are
 * the assembler's env_buffers / freq_buffers (asmparse.py:46-86 formats),
 * concatenated; channel c reads env words [env_off, env_off + env_len) and
 * freq words [freq_off, freq_off + freq_len).  Output: iq[c][n_samples] of
 * int16 {I, Q} pairs; sample j is at emulated cycle j / spc.
 *
 * The dpemu_dds_channels arrays are HOST memory (n_channels entries each);
 * summary / events / env_tables / freq_tables / iq_out are device pointers.
 * n_samples must be a multiple of 4; event_cap <= 1024.
 */
typedef struct dpemu_dds_channels {
    uint32_t n_channels;
    uint32_t n_lanes;          /* stride of the event arrays (dpemu_run's n_lanes) */
    uint32_t n_samples;        /* samples per channel                               */
    uint32_t event_cap;        /* event slots per lane of the event arrays          */
    const uint32_t *ch_lane;   /* lane of each channel                               */
    const uint32_t *ch_elem;   /* element (cfg & 3) of each channel                  */
    const uint32_t *spc;       /* samples per clock, 1..16                           */
    const uint32_t *interp;    /* output samples per envelope sample, >= 1           */
    const uint32_t *env_off;
    const uint32_t *env_len;
    const uint32_t *freq_off;
    const uint32_t *freq_len;
} dpemu_dds_channels;

int dpemu_dds(dpemu_ctx *ctx, const dpemu_dds_channels *ch, const uint32_t *summary,
              const uint32_t *events, const uint32_t *env_tables, const uint32_t *freq_tables,
              int16_t *iq_out, void *stream);

/* The Q15 sine table both the DDS kernel and its CPU restatement use. */
int dpemu_dds_sin_lut(int16_t *out4096);

/*
 * Measurement.  While kernel timing is on, dpemu_run and dpemu_dds record a
 * HIP event pair on the call's stream around their main kernel (the
 * interpreter / the DDS kernel; not the histogram memset and reduction).
 * dpemu_kernel_times waits for the recorded pairs, writes up to max_n
 * elapsed times in ms (oldest first) to ms, *n_out = how many, and clears the
 * record.  dpemu_last_kernel names the interpreter variant the last dpemu_run
 * launched (e.g. "straight_kernel<rows,fb1>", "macro_kernel", "interp_kernel<feat=0x3>").
 */
int         dpemu_set_kernel_timing(dpemu_ctx *ctx, int enable);
int         dpemu_kernel_times(dpemu_ctx *ctx, float *ms, int max_n, int *n_out);
const char *dpemu_last_kernel(dpemu_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* DPEMU_H */
