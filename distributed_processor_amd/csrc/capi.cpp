// capi.cpp -- the extern "C" boundary of libdpemu.so (include/dpemu.h).
//
// Replaces the reference's simulation harness: where the
// cocotb testbench loaded cmd_mem word by word (cocotb/proc/test_proc.py:29-38)
// and clocked one Verilator toplevel_sim, dpemu_load_programs uploads every
// assembled program once and dpemu_run executes n_shots x C cores on the GPU.
// Kernel choice depends only on the loaded programs, the grid size and the
// caller's exec_flags -- never on the environment.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.h"
#include "lds_grants.h"

using namespace dpemu;

namespace dpemu {
static LdsGrants g_lds_grants;     // the process's dynamic-LDS opt-ins, per (device, kernel)

hipError_t opt_in_dynamic_lds(const void *fn, size_t bytes)
{
    if (bytes <= LdsGrants::DEFAULT_LIMIT) return hipSuccess;
    int dev = 0;
    const hipError_t de = hipGetDevice(&dev);
    if (de != hipSuccess) return de;
    return (hipError_t)g_lds_grants.ensure(dev, fn, bytes, [&] {
        return (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    });
}
}  // namespace dpemu

struct dpemu_ctx {
    int device = 0;
    uint32_t n_cu = 256;                    // compute units of the device (hipDeviceAttributeMultiprocessorCount)
    std::string err;
    // programs
    uint4 *d_uops = nullptr;                // decode_cmd words, program-major (KParams::uops)
    uint4 *d_uops_t = nullptr;              // command-major copy (KParams::fetch), or null
    uint4 *d_macro = nullptr;               // macro image of branch-free ALU programs (macro.hip), or null
    uint32_t *d_moff = nullptr;             // its per-program offsets (in macros)
    uint32_t *d_mchunk = nullptr, *d_mcoff = nullptr;   // lean chunks (mark_lean_chunks) and their offsets
    uint32_t *d_offsets = nullptr, *d_ninstr = nullptr, *d_table = nullptr;
    uint32_t n_programs = 0, n_groups = 0, C = 0;
    bool has_fproc = false, has_sync = false, straight = false, linear = false, reg_writes = false;
    // register slots of the macro image (remap_macro_regs): 2 in VGPRs, else 16 (identity map)
    int macro_nr = 16;
    bool macro_addid = false;               // every ALU slot of the macro image is id0 / add
    bool macro_w3 = false;                  // the macro image has three ALU slots (kernels.h MACRO_W3)
    uint32_t macro_rs = 0;                  // UOP_RS_* fields its pulse slots register-source
    uint64_t reg_map = 0xFEDCBA9876543210ull, reg_inv = 0xFEDCBA9876543210ull;
    uint32_t reg_used = 0xFFFFu;
    uint32_t max_len = 0;              // longest program (commands)
    std::vector<uint64_t> group_len;   // instructions of all C programs of each group
    // DEMOD frequency tables (dpemu_load_readout_freqs), per loaded program
    uint32_t *d_ro_fq = nullptr;
    uint4 *d_ro_hdr = nullptr;
    // run constants: p1 thresholds [64] then DEMOD axes [64]
    uint32_t *d_thr = nullptr;
    uint64_t *d_lut = nullptr;
    std::vector<uint32_t> thr_cache;
    std::vector<uint64_t> lut_cache;
    // DDS
    int16_t *d_sin = nullptr;
    uint32_t *d_ch = nullptr;
    uint32_t ch_cap = 0;
    std::vector<uint32_t> ch_cache;
    void *d_dds_index = nullptr;            // event index of dds_index_kernel
    uint64_t dds_index_cap = 0;
    std::string last_kernel;                // variant the last dpemu_run launched (dpemu_last_kernel)
    // kernel timing (dpemu_set_kernel_timing): event pairs recorded around main kernels
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
    // privatised outcome histograms (R replicas, reduced after the interpreter)
    uint32_t *d_hist_rep = nullptr;
    uint64_t hist_rep_bytes = 0;
    bool hist_rep_dirty = true;     // replicas not known to be zero
    // call ordering across streams: the last call's stream and an event after its work
    hipEvent_t ord_ev = nullptr;
    hipStream_t ord_stream = nullptr;
    bool ord_valid = false;
};

static int fail(dpemu_ctx *ctx, int code, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
static int fail(dpemu_ctx *ctx, int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define HIPCHK(ctx, call)                                                                  \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(ctx, DPEMU_E_DEVICE, "%s: %s", #call, hipGetErrorString(e_));      \
    } while (0)

// Work of one context runs in call order whatever the streams: a call on a
// stream other than the previous call's first waits for the previous call's
// work (the scratch buffers -- histogram replicas, DDS index, thresholds, LUT
// table, channel descriptors -- are shared by the context's calls).
static hipError_t order_begin(dpemu_ctx *ctx, hipStream_t s)
{
    if (ctx->ord_valid && s != ctx->ord_stream) return hipStreamWaitEvent(s, ctx->ord_ev, 0);
    return hipSuccess;
}

static hipError_t order_end(dpemu_ctx *ctx, hipStream_t s)
{
    const hipError_t e = hipEventRecord(ctx->ord_ev, s);
    ctx->ord_stream = s;
    ctx->ord_valid = e == hipSuccess;
    return e;
}

// kernel timing: record the start event of a main-kernel launch on `stream`;
// *stop gets the pair's stop event (null while timing is off)
static hipError_t timing_start(dpemu_ctx *ctx, hipStream_t stream, hipEvent_t *stop)
{
    *stop = nullptr;
    if (!ctx->timing) return hipSuccess;
    std::pair<hipEvent_t, hipEvent_t> e;
    if (!ctx->ev_free.empty()) {
        e = ctx->ev_free.back();
        ctx->ev_free.pop_back();
    } else {
        hipError_t r = hipEventCreate(&e.first);
        if (r != hipSuccess) return r;
        r = hipEventCreate(&e.second);
        if (r != hipSuccess) { (void)hipEventDestroy(e.first); return r; }
    }
    ctx->ev_used.push_back(e);
    *stop = e.second;
    return hipEventRecord(e.first, stream);
}

// Macro image of a branch-free program (macro.hip): from its decoded
// commands u[0, n) (and the zero = DONE guard past the end), macros of up to
// `max_alu` consecutive reg_alu / inc_qclk commands followed by the next other
// command, until the first terminal command (done / 0000 / hang) -- the
// program's last macro, which the kernel re-reads once a lane has finished.
// Built WIDE, MACRO_WIDE u32 per macro: {imm, ctl} x 3 ALU slots then the
// pulse slot's decode_cmd word (w bit 31 = no command); ctl = present[31]
// inc_qclk[30] rs0[15:12] rd[11:8] rs1[7:4] in0_reg[3] alu_op[2:0].
// pack_macros turns it into the 32-B device image (kernels.h MACRO_W3).
constexpr uint32_t MACRO_WIDE = 10;
static void build_macros(const uint32_t *u, uint32_t n, uint32_t max_alu, std::vector<uint32_t> &out)
{
    static const uint32_t zero[4] = {0, 0, 0, 0};
    uint32_t k = 0;
    for (;;) {
        uint32_t m[MACRO_WIDE] = {0, 0, 0, 0, 0, 0, 0, 0, 0, MACRO_ABSENT};
        const uint32_t *c = k < n ? u + 4ull * k : zero;
        for (uint32_t a = 0; a < max_alu; a++) {
            const uint32_t op4 = c[1] >> 28;
            if (op4 != 0x1 && op4 != 0x6) break;
            m[2 * a] = c[0];
            m[2 * a + 1] = 0x80000000u | (op4 == 0x6 ? 0x40000000u : 0u) | (c[1] & 0xFFFu) | (((c[3] >> 20) & 15u) << 12);
            k++;
            c = k < n ? u + 4ull * k : zero;
        }
        const uint32_t op4 = c[1] >> 28;
        if (op4 != 0x1 && op4 != 0x6) {        // the slot's command (else: another ALU command opens the next macro)
            memcpy(m + 6, c, 16);
            k++;
        }
        out.insert(out.end(), m, m + MACRO_WIDE);
        if (op4 == 0x0 || op4 == 0xA || op4 >= 0xD) return;
    }
}

// ALU slot k's ctl of a packed macro (8 u32, macro.hip): legacy {imm0, ctl0,
// imm1, ctl1, pulse}, or MACRO_W3 {imm0, packed ctl, imm1, imm2, pulse}
static uint32_t macro_ctl(const uint32_t *m, int k, bool w3)
{
    if (!w3) return k < 2 ? m[2 * k + 1] : 0u;
    return w3_ctl(m[1], k);
}

// The 32-B device image from the wide one: MACRO_W3 packs three ALU slots
// (their ctl fields with 1-bit register slots, kernels.h w3_pack) when the
// image names at most 2 registers; else two slots, legacy layout.
static void pack_macros(const std::vector<uint32_t> &wide, bool w3, std::vector<uint32_t> &mac)
{
    const size_t n = wide.size() / MACRO_WIDE;
    mac.resize(8 * n);
    for (size_t i = 0; i < n; i++) {
        const uint32_t *w = &wide[MACRO_WIDE * i];
        uint32_t *m = &mac[8 * i];
        if (w3) {
            uint32_t pk = 0;
            for (int k = 0; k < 3; k++) pk |= w3_pack(w[2 * k + 1]) << (10 * k);
            m[0] = w[0]; m[1] = pk; m[2] = w[2]; m[3] = w[4];
        } else {
            m[0] = w[0]; m[1] = w[1]; m[2] = w[2]; m[3] = w[3];
        }
        memcpy(m + 4, w + 6, 16);
    }
}

// The reg_file registers the macro image names (ALU slot ctl: rs0 when
// in0_reg, rd and rs1 of reg_alu; pulse slot: rs0 when a field is
// register-sourced; an operand the ALU op ignores -- in1 of id0 / zero, in0
// of id1 / zero -- names nothing) renumbered to slots 0..n-1 in place when
// there are at most 2, so macro_staged_kernel keeps them in VGPRs.  Unnamed
// registers are never written and read as 0 (reg_file.v resets to 0); a
// field that names no register maps to slot 0 (its value is selected away).
// Returns the slot count (2, or 16 = left as is) and the maps
// (KParams::reg_map / reg_inv).
// registers the decode_cmd words u[0 .. n) name (the reg_file reads and
// writes of reg_alu / inc_qclk and the register-sourced pulse fields), by the
// rules remap_macro_regs applies to the macro image built from them
static uint32_t named_regs(const uint32_t *u, uint64_t n)
{
    uint32_t used = 0;
    for (uint64_t i = 0; i < n; i++, u += 4) {
        const uint32_t op4 = u[1] >> 28, rs0 = (u[3] >> 20) & 15u;
        if (op4 == 0x1u || op4 == 0x6u) {                      // reg_alu / inc_qclk
            const uint32_t op = u[1] & 7u;                      // alu.v: 0 id0, 6 id1, 7 zero
            if ((u[1] & 8u) && op != 6u && op != 7u) used |= 1u << rs0;
            if (op4 == 0x1u) {
                used |= 1u << ((u[1] >> 8) & 15u);
                if (op != 0u && op != 7u) used |= 1u << ((u[1] >> 4) & 15u);
            }
        } else if ((op4 == 0x8u || op4 == 0x9u) && (u[3] & UOP_ANY_RS)) {
            used |= 1u << rs0;
        }
    }
    return used;
}

static int remap_macro_regs(std::vector<uint32_t> &mac, uint64_t &map, uint64_t &inv, uint32_t &used)
{
    used = 0;
    for (size_t i = 0; i < mac.size(); i += MACRO_WIDE) {
        for (int a = 0; a < 3; a++) {
            const uint32_t ctl = mac[i + 2 * a + 1];
            if (!(ctl >> 31)) continue;
            const uint32_t op = ctl & 7u;                       // alu.v: 0 id0, 6 id1, 7 zero
            if ((ctl & 8u) && op != 6u && op != 7u) used |= 1u << ((ctl >> 12) & 15u);
            if (!((ctl >> 30) & 1u)) {
                used |= 1u << ((ctl >> 8) & 15u);
                if (op != 0u && op != 7u) used |= 1u << ((ctl >> 4) & 15u);
            }
        }
        const uint32_t w = mac[i + 9];
        if (!(w >> 31) && (w & UOP_ANY_RS)) used |= 1u << ((w >> 20) & 15u);
    }
    const int n = __builtin_popcount(used);
    if (n > 2) {
        map = inv = 0xFEDCBA9876543210ull;
        used = 0xFFFFu;
        return 16;
    }
    uint32_t slot[16] = {0};
    map = inv = 0;
    for (uint32_t r = 0, k = 0; r < 16; r++)
        if ((used >> r) & 1u) { slot[r] = k; map |= (uint64_t)k << (4 * r); inv |= (uint64_t)r << (4 * k); k++; }
    auto re = [&](uint32_t v, int sh) { return (v & ~(15u << sh)) | (slot[(v >> sh) & 15u] << sh); };
    for (size_t i = 0; i < mac.size(); i += MACRO_WIDE) {
        for (int a = 0; a < 3; a++) {
            uint32_t &ctl = mac[i + 2 * a + 1];
            if (ctl >> 31) ctl = re(re(re(ctl, 12), 8), 4);
        }
        uint32_t &w = mac[i + 9];
        if (!(w >> 31) && (w & UOP_ANY_RS)) w = re(w, 20);
    }
    return 2;
}

// Mark every macro of the lean-path shape (MACRO_SIMPLE, kernels.h) in the
// image's pulse slots, and return whether every ALU slot is reg_alu id0 / add
// (alu.v ops 0 / 1) and which pulse fields are register-sourced
static bool mark_simple_macros(std::vector<uint32_t> &mac, const std::vector<uint32_t> &moff, bool w3, uint32_t &rs)
{
    bool addid = true;
    rs = 0;
    size_t prog = 0;
    for (size_t m = 0, i = 0; i < mac.size(); i += 8, m++) {
        while (prog + 1 < moff.size() && moff[prog + 1] <= m) prog++;
        const bool first = moff[prog] == m;
        bool simple = !first;
        for (int a = 0; a < 3; a++) {
            const uint32_t ctl = macro_ctl(&mac[i], a, w3);
            if (!(ctl >> 31)) continue;
            if ((ctl >> 30) & 1u) simple = false;               // inc_qclk
            if ((ctl & 7u) > 1u) addid = false;
        }
        uint32_t &w = mac[i + 7];
        if (!(w >> 31)) {
            if ((mac[i + 5] >> 28) != 0x9u) simple = false;    // not PULSE_WRITE_TRIG
            rs |= w & (UOP_RS_ENV | UOP_RS_PH | UOP_RS_FR | UOP_RS_AMP);
        }
        if (simple) w |= MACRO_SIMPLE;
    }
    return addid;
}

// Per (program, chunk of MACRO_CHUNK macros as macro_staged_kernel stages
// them: macros [c CH, (c + 1) CH) of the program, the terminal macro
// repeating past its end): the largest pulse-slot cmd_time when every macro
// of the chunk is MACRO_SIMPLE and none is the terminal one (0 when no slot
// holds a pulse), else MACRO_CHUNK_MIXED.  A wave whose running lanes all
// hold such a chunk and can reach no max_cycles stop before its end runs the
// chunk's macros with no per-macro test (macro.hip lean_chunk_ok).
// chunk_off[p]: program p's first entry.
static void mark_lean_chunks(const std::vector<uint32_t> &mac, const std::vector<uint32_t> &moff,
                             std::vector<uint32_t> &chunk, std::vector<uint32_t> &chunk_off)
{
    const size_t n_prog = moff.size() - 1;
    chunk_off.resize(n_prog);
    chunk.clear();
    for (size_t pr = 0; pr < n_prog; pr++) {
        chunk_off[pr] = (uint32_t)chunk.size();
        const uint32_t nm = moff[pr + 1] - moff[pr];              // macros, the terminal one included
        for (uint32_t c = 0; c * MACRO_CHUNK < nm; c++) {
            uint32_t v = 0;
            if ((c + 1) * MACRO_CHUNK >= nm) v = MACRO_CHUNK_MIXED;  // reaches the terminal macro
            for (uint32_t j = 0; j < MACRO_CHUNK && v != MACRO_CHUNK_MIXED; j++) {
                const uint32_t *m = &mac[8ull * (moff[pr] + c * MACRO_CHUNK + j)];
                if (!(m[7] & MACRO_SIMPLE)) v = MACRO_CHUNK_MIXED;
                else if (!(m[7] >> 31)) v = std::max(v, m[4]);        // a pulse slot: its cmd_time
            }
            chunk.push_back(v);
        }
    }
}

static void free_programs(dpemu_ctx *ctx)
{
    for (void *q : {(void *)ctx->d_uops, (void *)ctx->d_uops_t, (void *)ctx->d_macro, (void *)ctx->d_moff,
                    (void *)ctx->d_mchunk, (void *)ctx->d_mcoff,
                    (void *)ctx->d_offsets, (void *)ctx->d_ninstr, (void *)ctx->d_table})
        (void)hipFree(q);
    ctx->d_uops = ctx->d_uops_t = ctx->d_macro = nullptr;
    ctx->d_mchunk = ctx->d_mcoff = nullptr;
    ctx->d_moff = ctx->d_offsets = ctx->d_ninstr = ctx->d_table = nullptr;
    ctx->n_programs = 0;
    (void)hipFree(ctx->d_ro_fq);
    (void)hipFree(ctx->d_ro_hdr);
    ctx->d_ro_fq = nullptr;
    ctx->d_ro_hdr = nullptr;
}

extern "C" {

int dpemu_abi_version(void) { return DPEMU_ABI_VERSION; }

int dpemu_struct_sizes(uint64_t *out)
{
    if (!out) return DPEMU_E_INVALID;
    out[0] = sizeof(dpemu_config);
    out[1] = sizeof(dpemu_outputs);
    out[2] = sizeof(dpemu_dds_channels);
    return DPEMU_OK;
}

int dpemu_create(int device, dpemu_ctx **out)
{
    if (!out) return DPEMU_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return DPEMU_E_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return DPEMU_E_DEVICE;
    dpemu_ctx *ctx = new dpemu_ctx();
    ctx->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        ctx->n_cu = (uint32_t)cus;
    std::vector<int16_t> lut(4096);
    dpemu_dds_sin_lut(lut.data());
    if (hipMalloc(&ctx->d_thr, 2 * DPEMU_MAX_CORES * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&ctx->d_lut, 256 * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&ctx->d_sin, 4096 * sizeof(int16_t)) != hipSuccess ||
        hipMemcpy(ctx->d_sin, lut.data(), 4096 * sizeof(int16_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ord_ev, hipEventDisableTiming) != hipSuccess) {
        dpemu_destroy(ctx);
        return DPEMU_E_NOMEM;
    }
    *out = ctx;
    return DPEMU_OK;
}

int dpemu_destroy(dpemu_ctx *ctx)
{
    if (!ctx) return DPEMU_E_INVALID;
    (void)hipSetDevice(ctx->device);
    if (ctx->ord_valid) (void)hipEventSynchronize(ctx->ord_ev);   // the context's work is done with its buffers
    free_programs(ctx);
    (void)hipFree(ctx->d_thr); (void)hipFree(ctx->d_lut); (void)hipFree(ctx->d_sin); (void)hipFree(ctx->d_ch);
    (void)hipFree(ctx->d_dds_index);
    (void)hipFree(ctx->d_hist_rep);
    for (auto *v : {&ctx->ev_used, &ctx->ev_free})
        for (auto &e : *v) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    if (ctx->ord_ev) (void)hipEventDestroy(ctx->ord_ev);
    delete ctx;
    return DPEMU_OK;
}

const char *dpemu_last_error(dpemu_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

const char *dpemu_last_kernel(dpemu_ctx *ctx) { return ctx ? ctx->last_kernel.c_str() : ""; }

int dpemu_set_kernel_timing(dpemu_ctx *ctx, int enable)
{
    if (!ctx) return DPEMU_E_INVALID;
    ctx->timing = enable != 0;
    return DPEMU_OK;
}

int dpemu_kernel_times(dpemu_ctx *ctx, float *ms, int max_n, int *n_out)
{
    if (!ctx || (max_n > 0 && !ms)) return DPEMU_E_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int n = 0;
    for (auto &e : ctx->ev_used) {
        HIPCHK(ctx, hipEventSynchronize(e.second));
        if (n < max_n) HIPCHK(ctx, hipEventElapsedTime(&ms[n], e.first, e.second));
        n++;
    }
    ctx->ev_free.insert(ctx->ev_free.end(), ctx->ev_used.begin(), ctx->ev_used.end());
    ctx->ev_used.clear();
    if (n_out) *n_out = n < max_n ? n : max_n;
    return DPEMU_OK;
}

int dpemu_load_programs(dpemu_ctx *ctx, const uint32_t *words, uint64_t n_cmds, const uint32_t *offsets,
                        const uint32_t *n_instr, uint32_t n_programs, const uint32_t *prog_table,
                        uint32_t n_groups, uint32_t cores_per_shot)
{
    if (!ctx) return DPEMU_E_INVALID;
    if ((!words && n_cmds) || !offsets || !n_instr || !prog_table || n_programs == 0 || n_groups == 0)
        return fail(ctx, DPEMU_E_INVALID, "load_programs: null array or empty program set");
    const uint32_t C = cores_per_shot;
    if (C == 0 || C > DPEMU_MAX_CORES || (C & (C - 1)))
        return fail(ctx, DPEMU_E_INVALID, "cores_per_shot %u is not a power of two in [1, 64]", C);
    if ((uint64_t)n_groups * C > 0xFFFFFFFFull) return fail(ctx, DPEMU_E_INVALID, "n_groups * C exceeds 2^32");
    bool fp = false, sy = false, straight = true, linear = true, rw = false;
    for (uint32_t i = 0; i < n_programs; i++) {
        if (n_instr[i] > 65536u)
            return fail(ctx, DPEMU_E_INVALID, "program %u: %u commands exceed the 2^16-deep cmd_mem", i, n_instr[i]);
        if ((uint64_t)offsets[i] + n_instr[i] > n_cmds)
            return fail(ctx, DPEMU_E_INVALID, "program %u: offset %u + %u commands run past the %llu commands",
                        i, offsets[i], n_instr[i], (unsigned long long)n_cmds);
    }
    for (uint32_t i = 0; i < n_programs; i++)
        for (uint32_t k = 0; k < n_instr[i]; k++) {
            const uint32_t op4 = words[4 * ((uint64_t)offsets[i] + k) + 3] >> 28;
            fp |= (op4 == 4 || op4 == 5);
            sy |= (op4 == 7);
            rw |= (op4 == 1 || op4 == 4);                  // reg_alu / alu_fproc write the reg_file
            straight &= !(op4 >= 1 && op4 <= 7);
            linear &= !(op4 >= 2 && op4 <= 5) && op4 != 7;     // no jump / fproc / sync: ip advances by 1
        }
    for (uint64_t i = 0; i < (uint64_t)n_groups * C; i++)
        if (prog_table[i] >= n_programs)
            return fail(ctx, DPEMU_E_INVALID, "prog_table[%llu] = %u >= n_programs", (unsigned long long)i, prog_table[i]);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (ctx->ord_valid) HIPCHK(ctx, hipEventSynchronize(ctx->ord_ev));   // earlier runs may still read the old image
    free_programs(ctx);
    HIPCHK(ctx, hipMalloc(&ctx->d_offsets, n_programs * 4));
    HIPCHK(ctx, hipMalloc(&ctx->d_ninstr, n_programs * 4));
    HIPCHK(ctx, hipMalloc(&ctx->d_table, (uint64_t)n_groups * C * 4));
    // every command pre-decoded once (kernels.h decode_cmd), program-major with
    // a zero (DONE) guard command after every program ...
    std::vector<uint32_t> goff(n_programs);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n_programs; i++) { goff[i] = (uint32_t)tot; tot += (uint64_t)n_instr[i] + 1; }
    if (tot >= (1ull << 32)) return fail(ctx, DPEMU_E_INVALID, "program set exceeds 2^32 commands");
    std::vector<uint32_t> uops(tot * 4, 0u);
    for (uint32_t i = 0; i < n_programs; i++)
        for (uint32_t k = 0; k < n_instr[i]; k++)
            decode_cmd(words + 4 * ((uint64_t)offsets[i] + k), &uops[4 * ((uint64_t)goff[i] + k)]);
    HIPCHK(ctx, hipMalloc(&ctx->d_uops, uops.size() * 4));
    HIPCHK(ctx, hipMemcpy(ctx->d_uops, uops.data(), uops.size() * 4, hipMemcpyHostToDevice));
    // ... and command-major (zero = DONE past a program's end, and one zero row
    // past the longest program for straight.hip) when the padding stays small:
    // at most 4x the programs, 1 GiB
    uint32_t max_len = 0;
    for (uint32_t i = 0; i < n_programs; i++) max_len = std::max(max_len, n_instr[i]);
    const uint64_t t_cmds = ((uint64_t)max_len + 1) * n_programs;
    if (max_len && t_cmds <= std::max<uint64_t>(4 * tot, 4096) && t_cmds * 16 <= (1ull << 30)) {
        std::vector<uint32_t> ut(t_cmds * 4, 0u);
        for (uint32_t pr = 0; pr < n_programs; pr++)
            for (uint32_t k = 0; k < n_instr[pr]; k++)
                memcpy(&ut[4 * ((uint64_t)k * n_programs + pr)], &uops[4 * ((uint64_t)goff[pr] + k)], 16);
        HIPCHK(ctx, hipMalloc(&ctx->d_uops_t, t_cmds * 16));
        HIPCHK(ctx, hipMemcpy(ctx->d_uops_t, ut.data(), t_cmds * 16, hipMemcpyHostToDevice));
    }
    // ... and the macro image of branch-free programs with register commands
    if (linear && !straight && max_len < 65536u) {
        // three ALU slots per macro when the image names at most 2 registers
        // (MACRO_W3: RB-like programs then have almost no macro without a
        // pulse, so a wave's programs stay on the same event slot and its
        // stores are whole rows), else two
        // the register count decides the layout before the image is built
        // (the guard commands are zero and name none)
        std::vector<uint32_t> wide, mac, moff(n_programs + 1);
        const bool w3 = __builtin_popcount(named_regs(uops.data(), tot)) <= 2;
        wide.reserve((tot * 4 + 8ull * n_programs) / 8 * MACRO_WIDE);
        for (uint32_t pr = 0; pr < n_programs; pr++) {
            moff[pr] = (uint32_t)(wide.size() / MACRO_WIDE);
            build_macros(&uops[4ull * goff[pr]], n_instr[pr], w3 ? 3u : 2u, wide);
            if (wide.size() / MACRO_WIDE >= (1ull << 32))
                return fail(ctx, DPEMU_E_INVALID, "macro image exceeds 2^32 macros");
        }
        moff[n_programs] = (uint32_t)(wide.size() / MACRO_WIDE);
        ctx->macro_nr = remap_macro_regs(wide, ctx->reg_map, ctx->reg_inv, ctx->reg_used);
        if ((ctx->macro_nr == 2) != w3)
            return fail(ctx, DPEMU_E_INVALID, "internal: macro register count disagrees with the decoded commands");
        ctx->macro_w3 = w3;
        pack_macros(wide, w3, mac);
        std::vector<uint32_t>().swap(wide);
        ctx->macro_addid = mark_simple_macros(mac, moff, w3, ctx->macro_rs);
        HIPCHK(ctx, hipMalloc(&ctx->d_macro, mac.size() * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_macro, mac.data(), mac.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMalloc(&ctx->d_moff, moff.size() * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_moff, moff.data(), moff.size() * 4, hipMemcpyHostToDevice));
        std::vector<uint32_t> mchunk, mcoff;
        mark_lean_chunks(mac, moff, mchunk, mcoff);
        HIPCHK(ctx, hipMalloc(&ctx->d_mchunk, mchunk.size() * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_mchunk, mchunk.data(), mchunk.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMalloc(&ctx->d_mcoff, mcoff.size() * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_mcoff, mcoff.data(), mcoff.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(ctx, hipMemcpy(ctx->d_offsets, goff.data(), n_programs * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->d_ninstr, n_instr, n_programs * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->d_table, prog_table, (uint64_t)n_groups * C * 4, hipMemcpyHostToDevice));
    ctx->n_programs = n_programs;
    ctx->n_groups = n_groups;
    ctx->C = C;
    ctx->has_fproc = fp;
    ctx->has_sync = sy;
    ctx->straight = straight;
    ctx->linear = linear;
    ctx->reg_writes = rw;
    ctx->max_len = max_len;
    ctx->group_len.assign(n_groups, 0);
    for (uint32_t g = 0; g < n_groups; g++)
        for (uint32_t c = 0; c < C; c++) ctx->group_len[g] += n_instr[prog_table[(uint64_t)g * C + c]] + 1;   // + guard
    return DPEMU_OK;
}

int dpemu_load_readout_freqs(dpemu_ctx *ctx, const uint32_t *words, uint64_t n_words, const uint32_t *drv_off,
                             const uint32_t *drv_len, const uint32_t *lo_off, const uint32_t *lo_len)
{
    if (!ctx) return DPEMU_E_INVALID;
    if (!ctx->n_programs) return fail(ctx, DPEMU_E_NOPROG, "load_readout_freqs before load_programs");
    if ((!words && n_words) || !drv_off || !drv_len || !lo_off || !lo_len)
        return fail(ctx, DPEMU_E_INVALID, "load_readout_freqs: null array");
    std::vector<uint32_t> hdr(4ull * ctx->n_programs);
    for (uint32_t i = 0; i < ctx->n_programs; i++) {
        if ((uint64_t)drv_off[i] + drv_len[i] > n_words || (uint64_t)lo_off[i] + lo_len[i] > n_words)
            return fail(ctx, DPEMU_E_INVALID, "load_readout_freqs: program %u's table runs past the %llu words", i,
                        (unsigned long long)n_words);
        hdr[4 * i] = drv_off[i]; hdr[4 * i + 1] = drv_len[i]; hdr[4 * i + 2] = lo_off[i]; hdr[4 * i + 3] = lo_len[i];
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (ctx->ord_valid) HIPCHK(ctx, hipEventSynchronize(ctx->ord_ev));   // earlier runs may still read the old tables
    (void)hipFree(ctx->d_ro_fq);
    (void)hipFree(ctx->d_ro_hdr);
    ctx->d_ro_fq = nullptr;
    ctx->d_ro_hdr = nullptr;
    HIPCHK(ctx, hipMalloc(&ctx->d_ro_fq, std::max<uint64_t>(n_words, 1) * 4));
    if (n_words) HIPCHK(ctx, hipMemcpy(ctx->d_ro_fq, words, n_words * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMalloc(&ctx->d_ro_hdr, hdr.size() * 4));
    HIPCHK(ctx, hipMemcpy(ctx->d_ro_hdr, hdr.data(), hdr.size() * 4, hipMemcpyHostToDevice));
    return DPEMU_OK;
}

static int validate(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t n_shots, bool want_hist)
{
    if (!cfg) return fail(ctx, DPEMU_E_INVALID, "null config");
    if (!ctx->n_programs) return fail(ctx, DPEMU_E_NOPROG, "run before load_programs");
    if (cfg->cores_per_shot != ctx->C)
        return fail(ctx, DPEMU_E_INVALID, "cores_per_shot %u != loaded %u", cfg->cores_per_shot, ctx->C);
    if (cfg->n_groups != ctx->n_groups)
        return fail(ctx, DPEMU_E_INVALID, "n_groups %u != loaded %u", cfg->n_groups, ctx->n_groups);
    if (cfg->shots_per_group == 0) return fail(ctx, DPEMU_E_INVALID, "shots_per_group == 0");
    if (cfg->n_groups > 0x80000000u) return fail(ctx, DPEMU_E_INVALID, "n_groups > 2^31");
    if (cfg->max_cycles == 0 || cfg->max_cycles > 0x7FFFFFC0u)
        return fail(ctx, DPEMU_E_INVALID, "max_cycles must be in (0, 2^31 - 64]");
    if (cfg->meas_latency < 1 || cfg->meas_latency > (1u << 20) || cfg->sync_latency < 1 ||
        cfg->sync_latency > (1u << 20))
        return fail(ctx, DPEMU_E_INVALID, "meas_latency / sync_latency must be in [1, 2^20]");
    if (cfg->meas_model > DPEMU_MEAS_DEMOD)
        return fail(ctx, DPEMU_E_INVALID, "meas_model must be DPEMU_MEAS_STATE, _READOUT or _DEMOD");
    if (cfg->meas_model == DPEMU_MEAS_DEMOD) {
        if (cfg->ro_drv_elem > 3 || cfg->ro_drv_elem == cfg->meas_elem)
            return fail(ctx, DPEMU_E_INVALID, "ro_drv_elem %u must be an element 0..3 other than meas_elem",
                        cfg->ro_drv_elem);
        if (cfg->ro_cpw < 1 || cfg->ro_cpw > DPEMU_RO_CPW_MAX)
            return fail(ctx, DPEMU_E_INVALID, "ro_cpw %u not in [1, %u]", cfg->ro_cpw, DPEMU_RO_CPW_MAX);
        if (cfg->ro_delay >= (1u << 20)) return fail(ctx, DPEMU_E_INVALID, "ro_delay must be < 2^20");
        if (cfg->ro_gain[0] > 65536 || cfg->ro_gain[1] > 65536)
            return fail(ctx, DPEMU_E_INVALID, "ro_gain must be <= 65536 (1.0 in Q16)");
        if (cfg->ro_sigma >= (1u << 24)) return fail(ctx, DPEMU_E_INVALID, "DEMOD: ro_sigma must be < 2^24");
        if ((uint64_t)cfg->max_cycles + cfg->meas_latency + 4096ull * DPEMU_RO_CPW_MAX + 64 >= 0x80000000ull)
            return fail(ctx, DPEMU_E_INVALID, "max_cycles + meas_latency + the readout window must stay below 2^31");
        if (!ctx->d_ro_hdr)
            return fail(ctx, DPEMU_E_INVALID, "DEMOD run without readout frequency tables (dpemu_load_readout_freqs)");
    }
    if (cfg->hist_assign > 1) return fail(ctx, DPEMU_E_INVALID, "hist_assign must be 0 or 1");
    if (cfg->lane_order > DPEMU_LANES_SHOT_MAJOR)
        return fail(ctx, DPEMU_E_INVALID, "lane_order %u is not DPEMU_LANES_CORE_MAJOR / SHOT_MAJOR", cfg->lane_order);
    if (cfg->ro_win >= 4096)
        return fail(ctx, DPEMU_E_INVALID, "ro_win %u must fit the 12-bit envelope-length field", cfg->ro_win);
    if ((uint64_t)cfg->max_cycles + cfg->meas_latency + 16 >= 0x80000000ull)
        return fail(ctx, DPEMU_E_INVALID, "max_cycles + meas_latency must stay below 2^31");
    if (cfg->meas_cap > 32) return fail(ctx, DPEMU_E_INVALID, "meas_cap > 32");
    if (cfg->event_cap > DPEMU_MAX_EVENT_CAP || cfg->trace_cap > DPEMU_MAX_EVENT_CAP)
        return fail(ctx, DPEMU_E_INVALID, "event_cap / trace_cap > %u", DPEMU_MAX_EVENT_CAP);
    if (cfg->fproc_mode > 1) return fail(ctx, DPEMU_E_INVALID, "fproc_mode %u", cfg->fproc_mode);
    if (cfg->lut_mask == 0) return fail(ctx, DPEMU_E_INVALID, "lut_mask must be nonzero");
    if (n_shots * cfg->cores_per_shot >= 0x80000000ull)
        return fail(ctx, DPEMU_E_INVALID, "n_shots * cores_per_shot must be < 2^31 per run");
    if (want_hist && cfg->cores_per_shot > 12)
        return fail(ctx, DPEMU_E_INVALID, "histogram needs cores_per_shot <= 12");
    return DPEMU_OK;
}

static int run_impl(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t shot_begin, uint64_t n_shots,
                    const dpemu_outputs *out, hipStream_t stream)
{
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, order_begin(ctx, stream));
    const uint32_t C = cfg->cores_per_shot;
    // run constants, uploaded when they change (stream-ordered: the copy lands
    // before this call's kernel and after the previous call's)
    std::vector<uint32_t> thr(cfg->p1_threshold, cfg->p1_threshold + DPEMU_MAX_CORES);
    thr.insert(thr.end(), cfg->ro_axis, cfg->ro_axis + DPEMU_MAX_CORES);   // d_thr[64..127]: DEMOD axes
    std::vector<uint64_t> lut(cfg->lut_table, cfg->lut_table + 256);
    if (thr != ctx->thr_cache) {
        ctx->thr_cache = thr;
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_thr, ctx->thr_cache.data(), thr.size() * 4, hipMemcpyHostToDevice, stream));
    }
    if (lut != ctx->lut_cache) {
        ctx->lut_cache = lut;
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_lut, ctx->lut_cache.data(), lut.size() * 8, hipMemcpyHostToDevice, stream));
    }
    KParams p{};
    p.uops = ctx->d_uops;
    const bool cmd_major = ctx->d_uops_t && !(cfg->exec_flags & DPEMU_X_PROG_MAJOR);
    p.fetch = cmd_major ? ctx->d_uops_t : ctx->d_uops;
    p.fetch_stride = cmd_major ? ctx->n_programs : 1u;
    p.offsets = ctx->d_offsets; p.n_instr = ctx->d_ninstr; p.prog_table = ctx->d_table;
    p.max_len = ctx->max_len;
    p.macros = ctx->d_macro; p.macro_off = ctx->d_moff;
    p.macro_chunk = ctx->d_mchunk; p.macro_coff = ctx->d_mcoff;
    p.reg_map = ctx->reg_map; p.reg_inv = ctx->reg_inv; p.reg_used = ctx->reg_used;
    p.macro_rs = ctx->macro_rs;
    p.macro_w3 = ctx->macro_w3 ? 1u : 0u;
    p.p1_thr = ctx->d_thr; p.lut_table = ctx->d_lut;
    p.summary = out->summary;
    p.events = reinterpret_cast<uint4 *>(out->events);
    p.trace = reinterpret_cast<uint4 *>(out->trace);
    p.meas = reinterpret_cast<uint2 *>(out->meas);
    p.regs_out = out->regs;
    p.hist = reinterpret_cast<unsigned long long *>(out->hist);
    p.hist_next = reinterpret_cast<unsigned long long *>(out->hist_next);
    p.hist_bins = (uint64_t)cfg->n_groups << C;
    p.shot_begin = shot_begin;
    p.n_lanes = (uint32_t)(n_shots * C);
    p.n_shots = (uint32_t)n_shots;
    p.shot_major = cfg->lane_order == DPEMU_LANES_SHOT_MAJOR;
    p.C = C;
    p.log2C = 0;
    while ((1u << p.log2C) < C) p.log2C++;
    p.n_groups = cfg->n_groups; p.shots_per_group = cfg->shots_per_group;
    p.grp_g0 = (uint32_t)((shot_begin / cfg->shots_per_group) % cfg->n_groups);
    p.grp_r0 = (uint32_t)(shot_begin % cfg->shots_per_group);
    fast_div_init(cfg->shots_per_group, p.spg_div);
    fast_div_init(cfg->n_groups, p.ng_div);
    p.max_cycles = cfg->max_cycles;
    p.event_cap = cfg->event_cap;           // the overflow flags follow the caps whether or not a buffer is given
    p.trace_cap = cfg->trace_cap;
    p.meas_cap = cfg->meas_cap;
    p.fproc_mode = cfg->fproc_mode; p.meas_elem = cfg->meas_elem;
    p.meas_latency = cfg->meas_latency; p.sync_latency = cfg->sync_latency;
    const uint64_t all = (C >= 64) ? ~0ull : ((1ull << C) - 1);
    p.sync_mask = cfg->sync_mask ? (cfg->sync_mask & all) : all;
    p.seed = cfg->seed;
    p.meas_model = cfg->meas_model; p.ro_sep = cfg->ro_sep; p.ro_thr = cfg->ro_thr; p.ro_sigma = cfg->ro_sigma;
    p.ro_win = cfg->ro_win;
    p.ro_wrecip = cfg->ro_win ? (1u << 24) / cfg->ro_win : 0u;
    p.ro_drv_elem = cfg->ro_drv_elem; p.ro_cpw = cfg->ro_cpw; p.ro_delay = cfg->ro_delay;
    p.ro_theta0 = cfg->ro_theta[0]; p.ro_theta1 = cfg->ro_theta[1];
    p.ro_gain0 = cfg->ro_gain[0]; p.ro_gain1 = cfg->ro_gain[1];
    p.ro_axis = ctx->d_thr + DPEMU_MAX_CORES;
    p.ro_fq = ctx->d_ro_fq; p.ro_hdr = ctx->d_ro_hdr;
    p.acc = reinterpret_cast<int2 *>(out->acc);
    p.lut_mask = cfg->lut_mask;
    const uint64_t guard = (uint64_t)C * (cfg->max_cycles / 3u + 4u) + 1024u;
    p.iter_guard = guard > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)guard;
    p.ev_stream = (cfg->exec_flags & DPEMU_X_STREAM_EVENTS) ? 1u : 0u;
    // LDS program staging: a workgroup of S = BLOCK / C shots spans at most w
    // consecutive program groups; stage their programs if they fit
    const uint32_t S = BLOCK / C, ng = cfg->n_groups;
    const uint64_t w = (ng == 1) ? 1 : (S - 1) / cfg->shots_per_group + 2;
    uint64_t footprint = ~0ull;
    if (w * C <= BLOCK) {
        const std::vector<uint64_t> &gl = ctx->group_len;
        uint64_t tot = 0;
        for (uint64_t x : gl) tot += x;
        footprint = (w / ng) * tot;
        const uint64_t r = w % ng;
        if (r) {
            uint64_t win = 0, best = 0;
            for (uint64_t i = 0; i < r; i++) win += gl[i % ng];
            best = win;
            for (uint64_t g = 1; g < ng; g++) {
                win += gl[(g + r - 1) % ng];
                win -= gl[g - 1];
                best = std::max(best, win);
            }
            footprint += best;
        }
    }
    p.prog_lds_words = 0;
    int feat = 0;
    // Pulse-only programs run on the wave-uniform-ip kernel (straight.hip)
    // unless ip could wrap (a 2^16-command program) or the general
    // interpreter is asked for (DPEMU_X_GENERAL).  Small grids (latency-bound)
    // fetch commands in batches of 4.  The kernel stages the workgroup's
    // programs in LDS when they fit the share of a CU's LDS that the grid's
    // co-resident workgroups leave and the programs are long (a dependent
    // global fetch per command is then the bottleneck); else it fetches the
    // command-major image.  The general interpreter stages only on request
    // (DPEMU_X_PROG_LDS), within 16 KiB.
    const uint64_t blocks = ((uint64_t)p.n_lanes + BLOCK - 1) / BLOCK;
    const bool small = blocks <= 4 * 256;
    const int fetch_batch = small ? 4 : 1;
    // the DEMOD readout model runs on branch_kernel<FEAT_DEMOD> (or the
    // general interpreter): the straight / macro kernels do not carry it
    const bool demod = cfg->meas_model == DPEMU_MEAS_DEMOD;
    const bool uniform = !demod && ctx->straight && ctx->max_len < 65536u && !(cfg->exec_flags & DPEMU_X_GENERAL);
    const bool macro = !demod && !uniform && ctx->d_macro && !(cfg->exec_flags & (DPEMU_X_GENERAL | DPEMU_X_PROG_LDS));
    // the staged macro kernel needs at most MACRO_SLOTS distinct programs per
    // wave: (program groups a wave's run of consecutive shots can span) x
    // (cores in the wave), for the thread mapping of block_core_major
    bool staged = false;
    uint32_t slots = 0;                     // program slots per wave of the staged kernel (0: macro_kernel)
    if (macro && !(cfg->exec_flags & DPEMU_X_MACRO_DIRECT)) {
        uint64_t shots_run, cores_w;
        if (cfg->lane_order == DPEMU_LANES_SHOT_MAJOR) {
            shots_run = std::max<uint64_t>(1, 64 / C);
            cores_w = std::min<uint64_t>(C, 64);
        } else {
            const uint64_t Sb = BLOCK / C;
            shots_run = std::min<uint64_t>(Sb, 64);
            cores_w = 64 / shots_run;
        }
        const uint64_t spg = cfg->shots_per_group;
        const uint64_t groups = ng == 1 ? 1 : std::min<uint64_t>(ng, (shots_run - 1 + spg - 1) / spg + 1);
        const uint64_t need = groups * cores_w;
        slots = need <= MACRO_SLOTS ? MACRO_SLOTS : (need <= MACRO_SLOTS_WIDE && ctx->macro_nr == 2) ? MACRO_SLOTS_WIDE : 0u;
        staged = slots != 0u;
    }
    int src = cmd_major ? STRAIGHT_ROWS : STRAIGHT_PROG;
    if (uniform) {
        const uint64_t per_cu = std::min<uint64_t>(8, std::max<uint64_t>(1, (blocks + 255) / 256));
        const uint64_t budget = std::min<uint64_t>(STRAIGHT_LDS_MAX, (150ull * 1024 / per_cu) / 16);
        if (footprint <= budget && ctx->max_len >= 64) {
            src = STRAIGHT_LDS;
            p.prog_lds_words = (uint32_t)std::max<uint64_t>(16, (footprint + 15) & ~15ull);
        }
    } else if (footprint <= PROG_LDS_MAX && (cfg->exec_flags & DPEMU_X_PROG_LDS)) {
        feat |= FEAT_PROG_LDS;
        p.prog_lds_words = (uint32_t)std::max<uint64_t>(16, (footprint + 15) & ~15ull);
    }
    if (ctx->has_fproc) feat |= (cfg->fproc_mode == DPEMU_FPROC_LUT) ? FEAT_LUT : FEAT_FPROC;
    if (ctx->has_sync) feat |= FEAT_SYNC;
    if (ctx->straight) feat |= FEAT_STRAIGHT;
    // outcome histogram.  Direct: one u64 atomic per shot into out->hist --
    // cheapest when concurrent shots spread over many bins.  Replicas: R
    // privatised u32 copies picked by workgroup, then a reduce kernel -- for
    // few bins hit by every wave at once (e.g. one program, 10^6 shots), where
    // direct atomics serialise on a few cache lines.  Default: replicas when
    // the bins a wave population touches concurrently are few.
    uint64_t bins = 0, hist_stride = 0;
    uint32_t R = 0;
    if (out->hist) {
        bins = (uint64_t)ng << C;
        const uint64_t spg = std::max<uint64_t>(1, cfg->shots_per_group);
        // groups live at once across ~64K resident lanes
        const uint64_t live_groups = std::min<uint64_t>(ng, (65536 / C) / spg + 1);
        bool repl = (live_groups << C) < 4096;
        if (cfg->exec_flags & DPEMU_X_HIST_DIRECT) repl = false;
        if (cfg->exec_flags & DPEMU_X_HIST_REPL) repl = true;
        p.hist_rep = nullptr;
        p.hist_lds = 0;
        if (repl) {
            const uint64_t stride = (bins + 31) & ~31ull;        // replicas on separate 128-B lines
            R = (uint32_t)std::min<uint64_t>({64, blocks, std::max<uint64_t>(1, (2ull << 20) / (stride * 4))});
            const uint64_t need = (uint64_t)R * stride * 4;
            if (need > ctx->hist_rep_bytes) {
                HIPCHK(ctx, hipStreamSynchronize(stream));    // earlier work may still use the old replicas
                (void)hipFree(ctx->d_hist_rep);
                ctx->d_hist_rep = nullptr; ctx->hist_rep_bytes = 0;
                HIPCHK(ctx, hipMalloc(&ctx->d_hist_rep, need));
                ctx->hist_rep_bytes = need;
                ctx->hist_rep_dirty = true;
            }
            // the reduce kernel leaves every replica word it read zero, so the
            // replicas are zeroed once per allocation (or after a failed run)
            if (ctx->hist_rep_dirty) {
                HIPCHK(ctx, hipMemsetAsync(ctx->d_hist_rep, 0, ctx->hist_rep_bytes, stream));
                ctx->hist_rep_dirty = false;
            }
            p.hist = nullptr;
            p.hist_rep = ctx->d_hist_rep;
            p.hist_reps = R;
            p.hist_stride = stride;
            p.hist_lds = bins <= HIST_LDS_MAX && (BLOCK / C) >= 4 * bins;   // LDS pre-aggregation pays
            hist_stride = stride;
        }
    }
    // branch.hip for every other program, the meas_lut back end included
    // (DPEMU_X_GENERAL / DPEMU_X_PROG_LDS: everything on the general
    // interpreter).  Its workgroup's programs are staged in LDS when they are
    // few commands: a fetch from LDS does not wait behind the lane's event
    // stores, which share vmcnt with global loads on gfx950
    // (DPEMU_X_PROG_MAJOR keeps the global fetch).
    const bool branch = !uniform && !macro && !(cfg->exec_flags & (DPEMU_X_GENERAL | DPEMU_X_PROG_LDS));
    int bfeat = (feat & (FEAT_FPROC | FEAT_LUT | FEAT_SYNC)) | (ctx->reg_writes ? FEAT_REGS : 0) |
                (demod ? FEAT_DEMOD : 0);
    if (branch) {
        p.prog_lds_words = 0;
        if (footprint <= BRANCH_LDS_MAX && !(cfg->exec_flags & DPEMU_X_PROG_MAJOR)) {
            bfeat |= FEAT_PROG_LDS;
            p.prog_lds_words = (uint32_t)std::max<uint64_t>(16, (footprint + 15) & ~15ull);
        }
    }
    if (out->hist && !p.hist_rep && cfg->hist_assign)      // direct atomics: assign = zero, then add
        HIPCHK(ctx, hipMemsetAsync(out->hist, 0, bins * sizeof(uint64_t), stream));
    // from the main launch until the reduce is enqueued the replicas may hold
    // counts: a failure in between leaves them to the next run's memset
    if (p.hist_rep) ctx->hist_rep_dirty = true;
    hipEvent_t ev_stop = nullptr;
    HIPCHK(ctx, timing_start(ctx, stream, &ev_stop));
    if (uniform) HIPCHK(ctx, launch_straight(p, src, fetch_batch, stream));
    else if (macro) HIPCHK(ctx, launch_macro(p, slots, ctx->macro_nr, ctx->macro_addid, stream));
    else if (branch) HIPCHK(ctx, launch_branch(p, bfeat, stream));
    else HIPCHK(ctx, launch_interp(p, feat, stream));
    if (ev_stop) HIPCHK(ctx, hipEventRecord(ev_stop, stream));
    {
        char name[96];
        if (uniform)
            snprintf(name, sizeof name, "straight_kernel<%s,fb%d>",
                     src == STRAIGHT_ROWS ? "rows" : src == STRAIGHT_PROG ? "prog" : "lds", fetch_batch);
        else if (macro && staged)
            snprintf(name, sizeof name, "macro_staged_kernel<%d%s%s>", ctx->macro_nr, ctx->macro_addid ? ",addid" : "",
                     slots > MACRO_SLOTS ? ",12" : "");
        else if (macro)
            snprintf(name, sizeof name, "macro_kernel");
        else if (branch)
            snprintf(name, sizeof name, "branch_kernel<feat=0x%x%s>", bfeat, C == 8 ? ",c8" : "");
        else
            snprintf(name, sizeof name, "interp_kernel<feat=0x%x>", feat);
        ctx->last_kernel = name;
    }
    if (out->hist && p.hist_rep) {
        HIPCHK(ctx, launch_hist_reduce(ctx->d_hist_rep, R, hist_stride, bins, cfg->hist_assign != 0,
                                       reinterpret_cast<unsigned long long *>(out->hist), stream));
        ctx->hist_rep_dirty = false;
    }
    HIPCHK(ctx, order_end(ctx, stream));
    return DPEMU_OK;
}

int dpemu_run(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t shot_begin, uint64_t n_shots,
              const dpemu_outputs *out, void *stream)
{
    if (!ctx) return DPEMU_E_INVALID;
    if (!out) return fail(ctx, DPEMU_E_INVALID, "null outputs");
    int rc = validate(ctx, cfg, n_shots, out->hist != nullptr || out->hist_next != nullptr);
    if (rc) return rc;
    if (out->acc && cfg->meas_model != DPEMU_MEAS_DEMOD)
        return fail(ctx, DPEMU_E_INVALID, "acc: DEMOD runs only");
    if (out->hist_next) {
        const uint64_t bytes = ((uint64_t)cfg->n_groups << cfg->cores_per_shot) * sizeof(uint64_t);
        const uintptr_t a = (uintptr_t)out->hist, b = (uintptr_t)out->hist_next;
        if (out->hist && a < b + bytes && b < a + bytes)
            return fail(ctx, DPEMU_E_INVALID, "hist_next overlaps hist");
        if (b % sizeof(uint64_t)) return fail(ctx, DPEMU_E_INVALID, "hist_next is not 8-byte aligned");
    }
    if (n_shots == 0) {
        if (out->hist_next) {                                // the contract holds for an empty run too,
            hipStream_t s = (hipStream_t)stream;             // in call order like any other call
            HIPCHK(ctx, hipSetDevice(ctx->device));
            HIPCHK(ctx, order_begin(ctx, s));
            HIPCHK(ctx, hipMemsetAsync(out->hist_next, 0,
                                       ((size_t)cfg->n_groups << cfg->cores_per_shot) * sizeof(uint64_t), s));
            HIPCHK(ctx, order_end(ctx, s));
        }
        return DPEMU_OK;
    }
    return run_impl(ctx, cfg, shot_begin, n_shots, out, (hipStream_t)stream);
}

int dpemu_run_host(dpemu_ctx *ctx, const dpemu_config *cfg, uint64_t shot_begin, uint64_t n_shots,
                   const dpemu_outputs *host_out)
{
    if (!ctx) return DPEMU_E_INVALID;
    if (!host_out) return fail(ctx, DPEMU_E_INVALID, "null outputs");
    if (host_out->hist_next) return fail(ctx, DPEMU_E_INVALID, "hist_next: device runs (dpemu_run) only");
    int rc = validate(ctx, cfg, n_shots, host_out->hist != nullptr);
    if (rc) return rc;
    if (host_out->acc && cfg->meas_model != DPEMU_MEAS_DEMOD)
        return fail(ctx, DPEMU_E_INVALID, "acc: DEMOD runs only");
    if (n_shots == 0) return DPEMU_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const uint64_t nl = n_shots * cfg->cores_per_shot;
    struct Buf { void *host; void *dev; size_t bytes; bool in; };
    Buf bufs[7] = {
        {host_out->summary, nullptr, nl * 32, false},
        {host_out->events, nullptr, (size_t)cfg->event_cap * nl * 16, false},
        {host_out->trace, nullptr, (size_t)cfg->trace_cap * nl * 16, false},
        {host_out->meas, nullptr, (size_t)cfg->meas_cap * nl * 8, false},
        {host_out->regs, nullptr, nl * 64, false},
        {host_out->hist, nullptr, (size_t)cfg->n_groups * (cfg->cores_per_shot <= 12 ? (1u << cfg->cores_per_shot) : 0) * 8, true},
        {host_out->acc, nullptr, (size_t)cfg->meas_cap * nl * 8, false},
    };
    int result = DPEMU_OK;
    for (auto &b : bufs) {
        if (!b.host || !b.bytes) { b.host = nullptr; continue; }
        if (hipMalloc(&b.dev, b.bytes) != hipSuccess) { result = fail(ctx, DPEMU_E_NOMEM, "device allocation of %zu bytes failed", b.bytes); break; }
        hipError_t e = b.in ? hipMemcpy(b.dev, b.host, b.bytes, hipMemcpyHostToDevice) : hipMemset(b.dev, 0, b.bytes);
        if (e != hipSuccess) { result = fail(ctx, DPEMU_E_DEVICE, "%s", hipGetErrorString(e)); break; }
    }
    if (result == DPEMU_OK) {
        dpemu_outputs d{};
        d.summary = (uint32_t *)bufs[0].dev; d.events = (uint32_t *)bufs[1].dev;
        d.trace = (uint32_t *)bufs[2].dev; d.meas = (uint32_t *)bufs[3].dev;
        d.regs = (uint32_t *)bufs[4].dev; d.hist = (uint64_t *)bufs[5].dev;
        d.acc = (int32_t *)bufs[6].dev;
        result = run_impl(ctx, cfg, shot_begin, n_shots, &d, nullptr);
        if (result == DPEMU_OK) {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) result = fail(ctx, DPEMU_E_DEVICE, "kernel: %s", hipGetErrorString(e));
        }
        for (auto &b : bufs)
            if (result == DPEMU_OK && b.host && b.dev &&
                hipMemcpy(b.host, b.dev, b.bytes, hipMemcpyDeviceToHost) != hipSuccess)
                result = fail(ctx, DPEMU_E_DEVICE, "copy back failed");
    }
    (void)hipDeviceSynchronize();
    for (auto &b : bufs) if (b.dev) (void)hipFree(b.dev);
    return result;
}

// Q15 sine table of the DDS: round(32767 sin(2 pi i / 4096)), built with integer-exact
// symmetry from the first quadrant so every build gets the same bytes.
int dpemu_dds_sin_lut(int16_t *out)
{
    if (!out) return DPEMU_E_INVALID;
    for (int i = 0; i <= 1024; i++) {
        const double v = std::round(32767.0 * std::sin(2.0 * M_PI * (double)i / 4096.0));
        const int16_t q = (int16_t)v;
        out[i & 4095] = q;                 // [0, pi/2]
        if (i < 1024) out[2048 - i] = q;   // (pi/2, pi]
        out[(2048 + i) & 4095] = (int16_t)-q;
        if (i < 1024 && i > 0) out[4096 - i] = (int16_t)-q;
    }
    return DPEMU_OK;
}

}  // extern "C"

extern "C" int dpemu_dds(dpemu_ctx *ctx, const dpemu_dds_channels *ch, const uint32_t *summary,
                         const uint32_t *events, const uint32_t *env_tables, const uint32_t *freq_tables,
                         int16_t *iq_out, void *stream)
{
    if (!ctx) return DPEMU_E_INVALID;
    if (!ch || !summary || !events || !env_tables || !freq_tables || !iq_out)
        return fail(ctx, DPEMU_E_INVALID, "dpemu_dds: null argument");
    if (ch->n_samples % 4) return fail(ctx, DPEMU_E_INVALID, "n_samples must be a multiple of 4");
    if (ch->event_cap > DDS_MAX_EVENTS) return fail(ctx, DPEMU_E_INVALID, "event_cap > %u", DDS_MAX_EVENTS);
    if (ch->n_channels == 0 || ch->n_samples == 0) return DPEMU_OK;
    if (ch->n_channels > 65535) return fail(ctx, DPEMU_E_INVALID, "n_channels > 65535");
    std::vector<uint32_t> desc((size_t)ch->n_channels * DDS_CH_WORDS);
    uint32_t env_max = 0, freq_max = 0;         // LDS staging sizes: largest tables that fit
    for (uint32_t i = 0; i < ch->n_channels; i++) {
        uint32_t *d = &desc[(size_t)i * DDS_CH_WORDS];
        d[0] = ch->ch_lane[i]; d[1] = ch->ch_elem[i] & 3u; d[2] = ch->spc[i]; d[3] = ch->interp[i];
        d[4] = ch->env_off[i]; d[5] = ch->env_len[i]; d[6] = ch->freq_off[i]; d[7] = ch->freq_len[i];
        if (d[0] >= ch->n_lanes) return fail(ctx, DPEMU_E_INVALID, "channel %u: lane %u >= n_lanes", i, d[0]);
        if (d[2] < 1 || d[2] > 16) return fail(ctx, DPEMU_E_INVALID, "channel %u: spc %u not in [1, 16]", i, d[2]);
        if (d[3] < 1) return fail(ctx, DPEMU_E_INVALID, "channel %u: interp must be >= 1", i);
        // staged words: (E, E') pairs for interp 1 (swizzled chunks), (R, R') pairs of the freq entries
        const uint32_t ew = d[3] == 1 ? dds_env_pairs_words(d[5]) : d[5], fw = 2 * d[7];
        if (ew <= DDS_ENV_LDS_MAX) env_max = std::max(env_max, ew);
        if (fw <= DDS_FREQ_LDS_MAX) freq_max = std::max(freq_max, fw);
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, order_begin(ctx, s));
    if (desc != ctx->ch_cache) {            // descriptors change rarely: upload only then
        HIPCHK(ctx, hipStreamSynchronize(s));   // an earlier launch may still read d_ch
        if (desc.size() > ctx->ch_cap) {
            (void)hipFree(ctx->d_ch);
            ctx->d_ch = nullptr; ctx->ch_cap = 0;
            HIPCHK(ctx, hipMalloc(&ctx->d_ch, desc.size() * 4));
            ctx->ch_cap = desc.size();
        }
        HIPCHK(ctx, hipMemcpy(ctx->d_ch, desc.data(), desc.size() * 4, hipMemcpyHostToDevice));
        ctx->ch_cache = desc;
    }
    DDSParams p{};
    p.summary = summary;
    p.events = reinterpret_cast<const uint4 *>(events);
    p.env = env_tables; p.freq = freq_tables;
    p.sin_lut = ctx->d_sin;
    p.ch = ctx->d_ch;
    p.iq = reinterpret_cast<uint32_t *>(iq_out);
    p.n_channels = ch->n_channels; p.n_lanes = ch->n_lanes; p.n_samples = ch->n_samples;
    p.event_cap = ch->event_cap;
    p.ev_lds = std::max<uint32_t>(8, (ch->event_cap + 7) & ~7u);
    p.env_lds = (env_max + 3) & ~3u;
    p.freq_lds = (freq_max + 3) & ~3u;
    p.tiles = (uint32_t)(((uint64_t)p.n_samples + DDS_TILE - 1) / DDS_TILE);
    auto stripe_plan = [&](uint32_t per_stripe) {
        p.stripes = std::max<uint32_t>(1, (p.tiles + per_stripe - 1) / per_stripe);
        p.wg_tiles = (p.tiles + p.stripes - 1) / p.stripes;
        return dds_lds_bytes(0, p.wg_tiles, p.env_lds, p.freq_lds);
    };
    {
        const uint32_t fixed = stripe_plan(DDS_TILES_PER_STRIPE);
        const uint32_t fit = fixed < DDS_WG_LDS_BUDGET ? (DDS_WG_LDS_BUDGET - fixed) / 20 & ~7u : 0u;
        p.rec_lds = std::min(p.ev_lds, std::max(fit, DDS_REC_LDS_MIN));
        if (p.rec_lds < p.ev_lds) {
            // dense channels: stage every record under the larger budget, with
            // more tiles per workgroup to spread its larger prologue
            if (stripe_plan(DDS_TILES_PER_STRIPE_DENSE) + p.ev_lds * 20 <= (uint32_t)DDS_WG_LDS_DENSE)
                p.rec_lds = p.ev_lds;
            else
                stripe_plan(DDS_TILES_PER_STRIPE);
        }
    }
    const uint64_t need = dds_index_bytes(p.n_channels, p.ev_lds);
    if (need > ctx->dds_index_cap) {         // the event index (grown, never shrunk)
        HIPCHK(ctx, hipStreamSynchronize(s));   // an earlier launch may still use it
        (void)hipFree(ctx->d_dds_index);
        ctx->d_dds_index = nullptr; ctx->dds_index_cap = 0;
        HIPCHK(ctx, hipMalloc(&ctx->d_dds_index, need));
        ctx->dds_index_cap = need;
    }
    uint8_t *b = static_cast<uint8_t *>(ctx->d_dds_index);
    p.xs = reinterpret_cast<uint4 *>(b);
    p.xr = reinterpret_cast<uint32_t *>(b + (uint64_t)p.n_channels * p.ev_lds * 16);
    p.cnt = reinterpret_cast<uint2 *>(b + (uint64_t)p.n_channels * p.ev_lds * 20);
    // channels 2i and 2i + 1 on one lane (a qdrv / rdrv pair per core, say): one
    // index workgroup loads that lane's events once for both
    p.pair_lanes = p.n_channels % 2 == 0;
    for (uint32_t i = 0; p.pair_lanes && i < p.n_channels; i += 2)
        p.pair_lanes = desc[(size_t)i * DDS_CH_WORDS] == desc[(size_t)(i + 1) * DDS_CH_WORDS];
    hipEvent_t ev_stop = nullptr;
    HIPCHK(ctx, launch_dds_index(p, s));   // outside the timed bracket: it holds the synthesis kernel alone
    HIPCHK(ctx, timing_start(ctx, s, &ev_stop));
    HIPCHK(ctx, launch_dds(p, s));
    if (ev_stop) HIPCHK(ctx, hipEventRecord(ev_stop, s));
    HIPCHK(ctx, order_end(ctx, s));
    return DPEMU_OK;
}
