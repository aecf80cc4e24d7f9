// kernels.h -- device-side parameter blocks and launchers of libdpemu.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dpemu.h"

namespace dpemu {

constexpr uint32_t BLOCK = 256;                 // 4 wavefronts per workgroup
constexpr uint32_t MEAS_LOOKUP = DPEMU_MEAS_LOOKUP;
constexpr uint32_t LUT_FIRE_CAP = DPEMU_LUT_FIRE_CAP;

// exclusive block scan of v (BLOCK threads); returns the prefix, *total the sum
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *s_tmp, uint32_t *total)
{
    const uint32_t tid = threadIdx.x, wl = tid & 63, wv = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (wl >= (uint32_t)o) x += y;
    }
    if (wl == 63) s_tmp[wv] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < BLOCK / 64; k++) {
        const uint32_t t = s_tmp[k];
        off += (k < wv) ? t : 0u;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

// kernel specialisations, chosen per run from the opcodes the programs use
constexpr int FEAT_FPROC = 1;   // fproc_meas reads (ALU_FPROC / JUMP_FPROC)
constexpr int FEAT_SYNC = 2;    // SYNC barriers
constexpr int FEAT_LUT = 4;     // fproc_lut back end
constexpr int FEAT_PROG_LDS = 8; // the workgroup's programs staged in LDS (fits PROG_LDS_MAX)
constexpr int FEAT_STRAIGHT = 16; // only pulse / idle / done / hang opcodes: no register file
constexpr int FEAT_REGS = 32;   // branch.hip: some command writes the reg_file (reg_alu / alu_fproc)
constexpr int FEAT_DEMOD = 64;  // branch.hip: meas_model DPEMU_MEAS_DEMOD (lane.h demod_readout)
constexpr uint32_t PROG_LDS_MAX = 1024;   // commands (16 KiB) of dynamic LDS per workgroup
constexpr uint32_t BRANCH_LDS_MAX = 512;  // commands (8 KiB): branch.hip stages its programs up to this

constexpr uint32_t ST_DONE = DPEMU_ST_DONE, ST_MAX_CYCLES = DPEMU_ST_MAX_CYCLES;
constexpr uint32_t ST_HUNG_OPCODE = DPEMU_ST_HUNG_OPCODE, ST_DEADLOCK = DPEMU_ST_DEADLOCK;
constexpr uint32_t F_LATE = DPEMU_F_LATE, F_EVENT_OVF = DPEMU_F_EVENT_OVF;
constexpr uint32_t F_TRACE_OVF = DPEMU_F_TRACE_OVF, F_MEAS_OVF = DPEMU_F_MEAS_OVF;
constexpr uint32_t F_DOUBLE_STROBE = DPEMU_F_DOUBLE_STROBE, F_GUARD = DPEMU_F_GUARD;
constexpr uint32_t TRACE_QCLK_LOAD = DPEMU_TRACE_QCLK_LOAD, TRACE_QCLK_RST = DPEMU_TRACE_QCLK_RST;

// Pre-decoded command: dpemu_load_programs re-packs every 128-bit cmd_mem
// word (decode_cmd) so the interpreter reads fields at fixed 32-bit
// positions instead of slicing hdl/proc.sv:89-107's layout (the same 16
// bytes per command):
//   x  cmd_time (cmd[36:5]) for pulse / idle; ALU immediate in0 (cmd[119:88])
//   y  op4[31:28]; pulse writes: env[23:0] cfg[27:24] immediates (zero when the
//      field is not written or register-sourced); other ops: alu[2:0]
//      in0_reg[3] rs1[7:4] rd[11:8]
//   z  pulse writes: phase[16:0] freq[25:17] immediates (bits 31:26 zero);
//      other ops: target[15:0] fproc_id[23:16]
//   w  rs0[23:20] (cmd[119:116]); pulse writes: amp[15:0] immediate,
//      register-sourced env[16] phase[17] freq[18] amp[19], write enables
//      env[24] cfg[25] phase[26] freq[27] amp[28] (hdl/pulse_reg.sv:38-97),
//      any register-sourced field[29]
constexpr uint32_t UOP_RS_ENV = 1u << 16, UOP_RS_PH = 1u << 17, UOP_RS_FR = 1u << 18, UOP_RS_AMP = 1u << 19;
constexpr uint32_t UOP_ANY_RS = 1u << 29;

__host__ __device__ inline void decode_cmd(const uint32_t w[4], uint32_t u[4])
{
    const uint32_t op4 = w[3] >> 28;
    const uint32_t rs0 = (w[3] >> 20) & 15u;
    u[0] = (op4 == 0x9 || op4 == 0xC) ? ((w[0] >> 5) | (w[1] << 27)) : ((w[2] >> 24) | (w[3] << 8));
    u[1] = (op4 << 28) | ((w[3] >> 24) & 7u) | (((w[3] >> 27) & 1u) << 3) | (((w[2] >> 20) & 15u) << 4) |
           (((w[2] >> 16) & 15u) << 8);
    u[2] = ((w[2] >> 4) & 0xFFFFu) | (((w[1] >> 20) & 0xFFu) << 16);
    u[3] = rs0 << 20;
    if (op4 == 0x8 || op4 == 0x9) {
        const uint32_t env_i = ((w[2] >> 26) | (w[3] << 6)) & 0xFFFFFFu, ph_i = (w[2] >> 7) & 0x1FFFFu;
        const uint32_t fr_i = ((w[1] >> 28) | (w[2] << 4)) & 0x1FFu, amp_i = (w[1] >> 10) & 0xFFFFu;
        const uint32_t cfg_i = (w[1] >> 5) & 0xFu;
        const uint32_t env_we = (w[3] >> 19) & 1u, env_rs = (w[3] >> 18) & 1u;
        const uint32_t ph_we = (w[2] >> 25) & 1u, ph_rs = (w[2] >> 24) & 1u;
        const uint32_t fr_we = (w[2] >> 6) & 1u, fr_rs = (w[2] >> 5) & 1u;
        const uint32_t amp_we = (w[1] >> 27) & 1u, amp_rs = (w[1] >> 26) & 1u;
        const uint32_t cfg_we = (w[1] >> 9) & 1u;
        const uint32_t rs = (env_we & env_rs) | ((ph_we & ph_rs) << 1) | ((fr_we & fr_rs) << 2) | ((amp_we & amp_rs) << 3);
        u[1] = (op4 << 28) | (env_we && !env_rs ? env_i : 0u) | (cfg_we ? cfg_i << 24 : 0u);
        u[2] = (ph_we && !ph_rs ? ph_i : 0u) | (fr_we && !fr_rs ? fr_i << 17 : 0u);
        u[3] = (rs0 << 20) | (amp_we && !amp_rs ? amp_i : 0u) | (rs << 16) | (env_we << 24) | (cfg_we << 25) |
               (ph_we << 26) | (fr_we << 27) | (amp_we << 28) | ((rs ? 1u : 0u) << 29);
    }
}

// Division of a 32-bit n by a run constant d >= 1 without a divide sequence
// (Hacker's Delight 10-8, unsigned): l = ceil(log2 d), m = floor(2^32 (2^l -
// d) / d) + 1 < 2^32, q = (t + ((n - t) >> min(l, 1))) >> max(l - 1, 0) with
// t = mulhi(m, n); exact for every n < 2^32 (tests/test_capi.py checks the
// formula).  A runtime-divisor u32 division costs ~20 VALU per lane.
inline void fast_div_init(uint32_t d, uint32_t out[3])
{
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) l++;
    out[0] = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    out[1] = l < 1 ? l : 1u;
    out[2] = l > 1 ? l - 1 : 0u;
}

struct KParams {
    // programs, as decode_cmd words (16 B per command)
    const uint4 *uops;            // program-major: program p's command i at offsets[p] + i
    const uint4 *fetch;           // the image the loop fetches from: command i of program p at
    uint32_t fetch_stride;        //   i * fetch_stride + (stride 1 ? offsets[p] : p); stride = the
                                  //   program count selects the command-major copy (zero past a
                                  //   program's end), where adjacent lanes -- adjacent programs --
                                  //   fetch adjacent commands
    const uint32_t *offsets, *n_instr, *prog_table;   // uops: a zero guard command follows every program
    uint32_t max_len;             // longest program; the command-major image's guard row
    const uint4 *macros;          // macro.hip image: 2 x uint4 per macro (capi.cpp build_macros)
    const uint32_t *macro_off;    // [n_programs + 1]: program p's macros [macro_off[p], macro_off[p + 1])
    const uint32_t *macro_chunk;  // per (program, MACRO_CHUNK-macro chunk): the largest pulse cmd_time of a
                                  //   chunk whose macros are all MACRO_SIMPLE (0: no pulse), else
                                  //   MACRO_CHUNK_MIXED (capi.cpp mark_lean_chunks)
    const uint32_t *macro_coff;   // [n_programs]: program p's chunk c at macro_chunk[macro_coff[p] + c]
    uint64_t reg_map;             // macro image register slots: reg_file register r is slot (reg_map >> 4 r) & 15
    uint64_t reg_inv;             //   for r in the reg_used mask (others are never named: they read 0);
    uint32_t reg_used;            //   slot s holds register (reg_inv >> 4 s) & 15 (trace addresses)
    uint32_t macro_rs;            // UOP_RS_* fields some pulse slot of the macro image register-sources
    uint32_t macro_w3;            // the macro image is MACRO_W3 (three ALU slots; always with 2 register slots)
    const uint32_t *p1_thr;
    const uint64_t *lut_table;
    // outputs (device, nullable); lane L = core * n_shots + shot (core-major)
    uint32_t *summary;
    uint4 *events;                // {t, env | cfg << 24 | kind << 28, phase | freq << 17, amp}
    uint4 *trace;
    uint2 *meas;
    uint32_t *regs_out;
    unsigned long long *hist;
    // run
    uint64_t shot_begin;
    uint32_t n_lanes, n_shots, C, log2C, n_groups, shots_per_group;
    uint32_t shot_major;          // dpemu_config.lane_order: lane = shot * C + core (else core * n_shots + shot)
    uint32_t grp_g0, grp_r0;      // (shot_begin / spg) % n_groups, shot_begin % spg
    uint32_t spg_div[3], ng_div[3];   // FastDiv of shots_per_group / n_groups (shot_group)
    uint32_t max_cycles, event_cap, trace_cap, meas_cap;
    uint32_t fproc_mode, meas_elem, meas_latency, sync_latency;
    uint64_t sync_mask, seed;
    uint32_t lut_mask;
    uint32_t meas_model;          // DPEMU_MEAS_STATE / DPEMU_MEAS_READOUT (ro_*: include/dpemu.h)
    int32_t ro_sep, ro_thr;
    uint32_t ro_sigma, ro_win, ro_wrecip;   // ro_wrecip = floor(2^24 / ro_win)
    // DEMOD readout model (lane.h demod_readout): config fields, the per-core
    // axes, the frequency tables (dpemu_load_readout_freqs) and the acc output
    uint32_t ro_drv_elem, ro_cpw, ro_delay, ro_theta0, ro_theta1, ro_gain0, ro_gain1;
    const uint32_t *ro_axis;      // [64] Q15 I | Q << 16
    const uint32_t *ro_fq;        // frequency words
    const uint4 *ro_hdr;          // [n_programs] {drv_off, drv_len, lo_off, lo_len}
    int2 *acc;                    // dpemu_outputs.acc (nullable)
    uint32_t iter_guard;
    uint32_t ev_stream;           // DPEMU_X_STREAM_EVENTS: macro_staged_kernel's event rows nontemporal
    uint32_t prog_lds_words;      // dynamic LDS commands (FEAT_PROG_LDS)
    uint32_t *hist_rep;           // [hist_reps][hist_stride] u32 replicas (128-B aligned rows)
    uint32_t hist_reps, hist_lds; // hist_lds: n_groups << C <= HIST_LDS_MAX, aggregate in LDS
    uint64_t hist_stride;
    unsigned long long *hist_next;  // dpemu_outputs.hist_next (nullable): zeroed by the kernel
    uint64_t hist_bins;             // n_groups << C (hist_next's words)
};
constexpr uint32_t HIST_LDS_MAX = 1024;

hipError_t launch_hist_reduce(uint32_t *rep, uint32_t R, uint64_t stride, uint64_t bins, bool assign,
                              unsigned long long *hist, hipStream_t stream);

hipError_t launch_interp(const KParams &p, int feat, hipStream_t stream);
// pulse-only programs (straight.hip); src: where commands are fetched from;
// fb: commands fetched per batch (1 or 4)
enum { STRAIGHT_ROWS = 0, STRAIGHT_PROG = 1, STRAIGHT_LDS = 2 };
constexpr uint32_t STRAIGHT_LDS_MAX = 9216;   // commands (144 KiB) of dynamic LDS per workgroup
hipError_t launch_straight(const KParams &p, int src, int fb, hipStream_t stream);
// dynamic LDS above 64 KiB for kernel `fn` on the current device: the opt-in,
// recorded per (device, kernel) under a lock (capi.cpp, lds_grants.h)
hipError_t opt_in_dynamic_lds(const void *fn, size_t bytes);
// programs with jumps / fproc_meas / sync (branch.hip): FEAT_FPROC | FEAT_SYNC | FEAT_REGS | FEAT_PROG_LDS bits of feat
hipError_t launch_branch(const KParams &p, int feat, hipStream_t stream);
// branch-free programs with reg_alu / inc_qclk (macro.hip): macro_staged_kernel
// when every wave runs at most MACRO_SLOTS distinct programs (nr = the
// register slots the macro image names: 2, else 16 in LDS), or at most
// MACRO_SLOTS_WIDE with nr == 2, else macro_kernel (slots = 0)
constexpr uint32_t MACRO_SLOTS = 8;     // distinct programs per wave whose macros are staged in LDS
constexpr uint32_t MACRO_SLOTS_WIDE = 12;   // ... for runs whose waves span 9-12 programs (NR == 2 images)
constexpr uint32_t MACRO_CHUNK = 16;    // macros per program per staged chunk (8: 3.84-4.12 vs 3.60 ms)
// addid: every ALU slot of the image is reg_alu id0 / add (RB phase updates)
// slots: 0 = macro_kernel (per-lane fetch), else the staged kernel's program slots per wave
hipError_t launch_macro(const KParams &p, uint32_t slots, int nr, bool addid, hipStream_t stream);
constexpr uint32_t MACRO_ABSENT = 0x80000000u;   // pulse slot w bit 31: no command; ALU ctl bit 31: present
// pulse slot w bit 30 (capi.cpp mark_simple_macros): not a program's first
// macro, its ALU slots are reg_alu (no inc_qclk) and its pulse slot is a
// PULSE_WRITE_TRIG or absent -- the shape macro_staged_kernel retires on its
// lean path (runtime conditions permitting)
constexpr uint32_t MACRO_SIMPLE = 0x40000000u;
constexpr uint32_t MACRO_CHUNK_MIXED = 0xFFFFFFFFu;   // macro_chunk: not every macro MACRO_SIMPLE
// MACRO_W3 image (KParams::macro_w3; the image names at most 2 registers):
// THREE ALU slots in the same 32 B, {imm0, packed ctl, imm1, imm2} + pulse
// slot.  Slot k's ctl is the 9-bit field at bit 10 k: op[2:0] in0_reg[3]
// rs1[4] rd[5] rs0[6] inc_qclk[7] present[8] (register fields are slots 0 /
// 1 after capi.cpp remap_macro_regs).  w3_ctl expands a field to the legacy
// ctl layout (present[31] inc_qclk[30] rs0[15:12] rd[11:8] rs1[7:4]
// in0_reg[3] op[2:0]); w3_pack is its inverse on 1-bit register fields.
constexpr uint32_t W3_OP = 0, W3_IN0 = 3, W3_RS1 = 4, W3_RD = 5, W3_RS0 = 6, W3_INC = 7, W3_PRES = 8;
__host__ __device__ inline uint32_t w3_ctl(uint32_t packed, int k)
{
    const uint32_t f = packed >> (10 * k);
    return (f & 0x1Fu) | (((f >> W3_RD) & 1u) << 8) | (((f >> W3_RS0) & 1u) << 12) | (((f >> W3_INC) & 1u) << 30) |
           (((f >> W3_PRES) & 1u) << 31);
}
__host__ __device__ inline uint32_t w3_pack(uint32_t ctl)
{
    if (!(ctl >> 31)) return 0u;
    return (ctl & 0x1Fu) | (((ctl >> 8) & 1u) << W3_RD) | (((ctl >> 12) & 1u) << W3_RS0) |
           (((ctl >> 30) & 1u) << W3_INC) | (1u << W3_PRES);
}

// ---- DDS ------------------------------------------------------------------
// Two launches per synthesis (dds.hip): dds_index_kernel compacts each
// channel's strobes and pulse resets once and writes every sample tile's
// window of them; dds_tile_kernel, grid (DDS stripes, channels), sweeps the
// tiles of a channel round-robin over its stripe workgroups, so the
// workgroups of a channel write adjacent tiles at the same time.
struct DDSParams {
    const uint32_t *summary;
    const uint4 *events;           // dpemu_run event records, slot-major
    const uint32_t *env, *freq;
    const int16_t *sin_lut;        // Q15 sine table [4096]
    const uint32_t *ch;            // per-channel descriptors, DDS_CH_WORDS u32 each
    uint32_t *iq;                  // [n_channels][n_samples] packed {I16 low, Q16 high}
    uint32_t n_channels, n_lanes, n_samples, event_cap;
    uint32_t ev_lds;               // compacted-event slots per channel (>= event_cap, multiple of 8)
    uint32_t rec_lds;              // strobe records / reset times a tile workgroup stages in LDS (<= ev_lds)
    uint32_t env_lds, freq_lds;    // LDS staging capacity for a channel's env / freq table (words, as staged)
    uint32_t tiles;                // tile windows per channel (DDS_TILE samples each)
    uint32_t stripes;              // tile workgroups per channel
    uint32_t wg_tiles;             // most tiles one workgroup sweeps (its LDS window slots)
    // event index (dds_index_kernel -> dds_tile_kernel)
    uint4 *xs;                     // [n_channels][ev_lds] strobes {t, env word, phase | freq << 17, amp}
    uint32_t *xr;                  // [n_channels][ev_lds] pulse_reset times
    uint2 *cnt;                    // [n_channels] {strobes, resets}
    uint32_t pair_lanes;           // channels 2i, 2i + 1 share a lane (one index workgroup per pair)
};
constexpr uint32_t DDS_CH_WORDS = 8;   // lane, elem, spc, interp, env_off, env_len, freq_off, freq_len
constexpr uint32_t DDS_MAX_EVENTS = 1024;
constexpr uint32_t DDS_TILE = 4 * BLOCK;      // samples per tile: 4 per thread, one 16-B store each
// tiles per stripe workgroup: 8 / 12 / 20 / 24 / 32 measured 0.419 / 0.346 /
// 0.315 / 0.325 / 0.345 ms against 0.313 for 16 (config 5)
#ifndef DDS_TILES_PER_STRIPE
#define DDS_TILES_PER_STRIPE 16u
#endif
constexpr uint32_t DDS_ENV_LDS_MAX = 8192;    // words: tables up to 32 KiB are staged in LDS
constexpr uint32_t DDS_FREQ_LDS_MAX = 2048;   // words: 64 freq entries as (R, R') pairs

// dynamic LDS bytes of dds_tile_kernel: quarter sine table (entries
// 0..1031) | strobe records (16 B) | reset times | tile windows | env | freq |
// the cycle sweep's per-wave store transpose (1 KiB per wave)
constexpr uint32_t DDS_LUT_BYTES = 1032 * 2;
constexpr uint32_t DDS_XPOSE_BYTES = (BLOCK / 64) * 1024;
__host__ __device__ inline uint32_t dds_lds_bytes(uint32_t rec_lds, uint32_t tiles_per_stripe, uint32_t env_lds,
                                                  uint32_t freq_lds)
{
    return DDS_LUT_BYTES + rec_lds * 20 + tiles_per_stripe * 16 + (env_lds + freq_lds) * 4 + DDS_XPOSE_BYTES;
}
// LDS budget of a tile workgroup: 8 workgroups (32 waves, the VGPR-bound
// occupancy) share a CU's 160 KiB.  The record capacity is what is left of
// it (at least DDS_REC_LDS_MIN); a stripe whose window holds more strobes or
// resets than that reads them from the global index instead.
// (less 512 B: the compiler's static LDS of the kernel, so 8 fit in 160 KiB)
constexpr uint32_t DDS_WG_LDS_BUDGET = 20 * 1024 - 512;
constexpr uint32_t DDS_REC_LDS_MIN = 64;
// Dense channels (more strobes than the 20-KiB budget holds, e.g. depth-200
// two-qubit RB drive channels, ~560-720 strobes): every record is staged when
// the workgroup then stays within this larger budget (fewer workgroups per CU,
// but no sweep reading records from the global index)
#ifndef DDS_WG_LDS_DENSE
#define DDS_WG_LDS_DENSE (32 * 1024 - 512)
#endif
// tiles per stripe workgroup under the dense budget (5 workgroups per CU
// instead of 8): config 5 on the two-qubit RB timelines, 16 / 20 / 22 / 24 /
// 26 / 28 / 32 tiles: 0.892 / 0.809 / 0.795 / 0.780 / 0.785 / 0.859 / 0.861
// ms (profiles/r06_dds_dense_ab.json); the sparse case keeps 16
#ifndef DDS_TILES_PER_STRIPE_DENSE
#define DDS_TILES_PER_STRIPE_DENSE 24u
#endif

// LDS words of an interp-1 envelope of n words staged as swizzled (E, E')
// pairs (dds.hip env_pair): whole groups of 8 16-B chunks
__host__ __device__ inline uint32_t dds_env_pairs_words(uint32_t n) { return (2 * n + 31) & ~31u; }

// bytes of the event index (xs, xr, cnt)
inline uint64_t dds_index_bytes(uint32_t n_channels, uint32_t ev_lds)
{
    return (uint64_t)n_channels * ev_lds * 20 + (uint64_t)n_channels * 8;
}

hipError_t launch_dds_index(const DDSParams &p, hipStream_t stream);
hipError_t launch_dds(const DDSParams &p, hipStream_t stream);

}  // namespace dpemu
