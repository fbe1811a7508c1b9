// gsa_capi.hip -- extern "C" boundary of libgsa.so (declared in include/gsa.h).
//
// Device-resident entry points enqueue the wavefront fills (nw_krow.hip sparse, nw_lane.hip full,
// nw_strip.hip score-only and the GSA_SPARSE_KERNEL=strip fallback); host-buffer
// entry points reproduce what the reference's align functions do around their kernels
// (allocate, copy in, fill, copy out, Stopwatch laps):
//   NwAlign_Gpu3_Ml_DiagDiag        nwalign_gpu3_ml_diagdiag.cu:288-596     -> gsa_align_full
//   NwAlign_Gpu9_Mlsp_DiagDiagDiag  nwalign_gpu9_mlsp_diagdiagdiag.cu:368-722 -> gsa_align_sparse
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gsa.h"
#include "nw_bidi.h"
#include "nw_check.h"
#include "nw_lane.h"
#include "nw_expand.h"
#include "nw_krow.h"
#include "nw_strip.h"
#include "nw_trace_dev.h"
#include "nw_scan.h"

namespace gsa {
int fold_moves(const unsigned char* moves, int64_t n, char* edit, int64_t cap, int64_t* edit_len, uint32_t* trace_hash);
}

struct gsa_ctx
{
    int device = 0;
    int cu_count = 0;
    long long lds_max = 65536;  // dynamic LDS a workgroup may opt into (bytes)
    hipStream_t stream = nullptr;
    // [0] ticket (zeroed per launch), [1] error flags: sticky across launches, read and cleared
    // by gsa_sync (or by the synchronous call that reports them)
    unsigned* ctl = nullptr;
    unsigned long long spin_ticks = 100000000ull;  // watchdog: 1 s of s_memrealtime (100 MHz)
    unsigned long long* gran = nullptr;
    size_t gran_elems = 0;
    unsigned epoch = 0;
    int last_hip_error = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // scratch buffers for the host-buffer entry points (grow-only, like DeviceArray::init)
    void* dbuf[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t dcap[5] = {0, 0, 0, 0, 0};
    // pair descriptors of the last launches: device copy + pinned host staging slots, each
    // slot reused only after the event recorded behind its copy has completed
    gsa::PairDesc* desc = nullptr;
    size_t desc_cap = 0;
    static constexpr int kStage = 4;
    gsa::PairDesc* stage[kStage] = {nullptr, nullptr, nullptr, nullptr};
    size_t stage_cap[kStage] = {0, 0, 0, 0};
    hipEvent_t stage_ev[kStage] = {nullptr, nullptr, nullptr, nullptr};
    bool stage_used[kStage] = {false, false, false, false};
    int stage_next = 0;
    // two-pass full fill (nw_expand.h): pass-1 outputs (header rows / columns, rows 64m) of the
    // last launch, grow-only; the expansion's pair descriptors: device copy + pinned staging slots
    void* exbuf = nullptr;
    size_t excap = 0;
    void* exdesc = nullptr;
    size_t exdesc_cap = 0;
    // the split batch (enqueue_full_split): the tail group's pass-1 outputs and descriptors, its
    // high-priority stream and the events between the groups
    void* exbuf2 = nullptr;
    size_t excap2 = 0;
    void* exdesc2 = nullptr;
    size_t exdesc_cap2 = 0;
    hipStream_t splitstream = nullptr;
    hipEvent_t split_ev[2] = {nullptr, nullptr};
    // fused single-pair fill: one progress word per pass-1 strip (epoch-tagged, cleared once per
    // allocation)
    unsigned long long* xdone = nullptr;
    size_t xdone_cap = 0;
    // GSA_STAMPS=1: the fused fill's stamps of the last launch (gsa_debug_stamps)
    unsigned long long* stamps = nullptr;
    size_t stamps_cap = 0, stamps_n = 0;
    hipStream_t stamps_stream = nullptr;  // the stream of the launch that wrote them
    // gsa_set_full_timing: events around the passes of the last two-pass full fill and the
    // expansion's per-workgroup clock stamps
    bool timing = false;
    hipEvent_t pev[3] = {nullptr, nullptr, nullptr};
    unsigned long long* clk = nullptr;
    size_t clk_cap = 0, clk_n = 0;
    int timing_state = 0;  // 0 none, 1 two launches (events + stamps), 2 fused (one launch), 3 pipelined
    int timing_groups = 0;
    // the batch expansion's task order, tuned per output buffer (enqueue_full_twopass): key, the
    // order each candidate took (ms, < 0: not measured), the order of the last launch and its events
    struct XTune
    {
        const void* key = nullptr;
        int pairs = 0;
        long long tasks = 0;
        float ms[2] = {-1.f, -1.f};
        int last = -1;
        bool pending = false;
        bool cold = true;  // the first launch on a key runs untimed (fresh pages, first-touch costs)
        hipEvent_t ev[2] = {nullptr, nullptr};
    } xt[2];  // per scratch slot
    // a batch that can run as two pair groups (enqueue_full_split): whole-job times of the four
    // candidates (one group or two, expansion order 1 or 2), keyed by the batch (enqueue_full)
    struct FTune
    {
        uint64_t key = 0;
        float ms[4] = {-1.f, -1.f, -1.f, -1.f};
        int last = -1;
        bool pending = false;
        bool cold = true;  // the first launch on a key runs untimed (fresh pages, first-touch costs)
        hipEvent_t ev[2] = {nullptr, nullptr};
    } ft;
    // score-only NW from both ends (score_bidi): tap rows of both halves, the reversed sequences, the
    // combine's result, the transposed table
    int* bidi = nullptr;
    size_t bidi_cap = 0;  // ints
    void* expin[kStage] = {nullptr, nullptr, nullptr, nullptr};
    size_t expin_cap[kStage] = {0, 0, 0, 0};
    hipEvent_t expin_ev[kStage] = {nullptr, nullptr, nullptr, nullptr};
    bool expin_used[kStage] = {false, false, false, false};
    int expin_next = 0;
    unsigned long long* chk = nullptr;  // verification results (nw_check.hip)
    // device traceback (nw_trace_dev.hip): move bytes, [moves, cost], global move codes
    unsigned char* tmoves = nullptr;
    size_t tmoves_cap = 0;
    long long* tres = nullptr;
    unsigned* tdirs = nullptr;
    size_t tdirs_cap = 0;  // bytes
    // tiles precomputed around the diagonal (trace_band): codes, and [list | map] ints
    unsigned* tband = nullptr;
    size_t tband_cap = 0;  // bytes
    int* tlist = nullptr;
    size_t tlist_cap = 0;  // ints
    // score-only fills (nw_scan.hip): boundary rows H/F, progress words, control words
    int* sbnd = nullptr;
    size_t sbnd_cap = 0;  // ints
    // mlsppt: host-mapped per-tile-row words (epoch << 32 | column chunks in memory); a pinned
    // host buffer the strided column chunks are packed into by a kernel on ptstream
    unsigned long long* ptflags = nullptr;
    void* ptpin = nullptr;  // pinned host memory (hipHostMallocDefault), ptpin_cap bytes (>= kPtPin)
    size_t ptpin_cap = 0;
    hipEvent_t ptev[2] = {nullptr, nullptr};
    static constexpr size_t kPtPin = 64u << 20;  // two slots
    hipStream_t ptstream = nullptr;
    size_t ptflags_cap = 0;
    // score-only control words: row scan [0] ticket|err, [1] best key, [2] result; AG/SW strip
    // [0] result, [1] best key, [3] its own error word (the fills' sticky word is not touched)
    unsigned long long* sctl = nullptr;
    // copy-back of the host-buffer entry points into pageable caller memory: per copy thread a
    // stream and two pinned chunks (DMA of chunk k+1 overlaps the host copy of chunk k)
    static constexpr int kCopyThreads = 8;
    static constexpr size_t kCopyChunk = 4u << 20;
    hipStream_t xstream[kCopyThreads] = {};
    void* xstage[kCopyThreads][2] = {};
    hipEvent_t xev[kCopyThreads][2] = {};
    gsa_mem_stats mem {};  // peak resource use of the fills since creation / gsa_mem_stats_reset
    // phase-boundary callback of the host-buffer entry points (gsa_set_lap_callback)
    gsa_lap_fn lap_fn = nullptr;
    void* lap_user = nullptr;
    // the knobs (kKnobNames): the environment when the context was created, then gsa_set_knob
    std::map<std::string, std::string> knobs;
};

namespace {

using Clock = std::chrono::steady_clock;

inline float ms_since(Clock::time_point& t)
{
    auto now = Clock::now();
    float ms = std::chrono::duration<float, std::milli>(now - t).count();
    t = now;
    return ms;
}

// Phase boundary of a host-buffer entry point: the caller's Stopwatch::lap(name)
// (stopwatch.cpp:43-50) through the registered callback, at the points the reference's align
// functions lap (nwalign_gpu9_mlsp_diagdiagdiag.cu:459-719)
inline void lap(gsa_ctx* ctx, const char* name)
{
    if (ctx->lap_fn) ctx->lap_fn(ctx->lap_user, name);
}

inline int fail(gsa_ctx* ctx, hipError_t e, int stat)
{
    ctx->last_hip_error = (int)e;
    return stat;
}

int ensure_dev(gsa_ctx* ctx, int slot, size_t bytes)
{
    if (ctx->dcap[slot] >= bytes && ctx->dbuf[slot]) return GSA_SUCCESS;
    if (ctx->dbuf[slot]) (void)hipFree(ctx->dbuf[slot]);
    ctx->dbuf[slot] = nullptr;
    ctx->dcap[slot] = 0;
    hipError_t e = hipMalloc(&ctx->dbuf[slot], std::max<size_t>(bytes, 256));
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    ctx->dcap[slot] = std::max<size_t>(bytes, 256);
    return GSA_SUCCESS;
}

int ensure_gran(gsa_ctx* ctx, size_t elems, hipStream_t st)
{
    if (ctx->gran_elems >= elems && ctx->gran) return GSA_SUCCESS;
    if (ctx->gran) (void)hipFree(ctx->gran);
    ctx->gran = nullptr;
    ctx->gran_elems = 0;
    hipError_t e = hipMalloc(&ctx->gran, elems * sizeof(unsigned long long));
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    // tags must never match a live epoch by accident: clear once per allocation, in stream order
    // before the launch that uses it (a non-blocking stream is not ordered behind the null stream)
    e = hipMemsetAsync(ctx->gran, 0, elems * sizeof(unsigned long long), st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    ctx->gran_elems = elems;
    return GSA_SUCCESS;
}

int ensure_desc(gsa_ctx* ctx, size_t n)
{
    if (ctx->desc_cap >= n && ctx->desc) return GSA_SUCCESS;
    if (ctx->desc) (void)hipFree(ctx->desc);
    ctx->desc = nullptr;
    ctx->desc_cap = 0;
    const size_t cap = std::max<size_t>(n, 64);
    hipError_t e = hipMalloc(&ctx->desc, cap * sizeof(gsa::PairDesc));
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    ctx->desc_cap = cap;
    return GSA_SUCCESS;
}

int check_inputs(int32_t adjrows, int32_t adjcols, int32_t substsz)
{
    if (adjrows < 1 || adjcols < 1) return GSA_ERROR_INVALID_VALUE;
    if (substsz < 1 || substsz > 32) return GSA_ERROR_INVALID_VALUE;  // LDS profile holds <= 32 letters
    return GSA_SUCCESS;
}

// Knobs: measurement and test switches, named as environment variables.  A context reads them
// once, from the environment, when it is created (gsa_ctx_create); gsa_set_knob changes them per
// context.  Launches never read the environment.
constexpr const char* kKnobNames[] = {
    "GSA_SPARSE_KERNEL", "GSA_KROW_K",      "GSA_KROW_NS",      "GSA_KROW_Q8",       "GSA_LANE_NS",
    "GSA_LANE_FEED",     "GSA_LANE_PAIR",   "GSA_FULL_KERNEL",  "GSA_FULL_FUSED",    "GSA_FULL_SPLIT",
    "GSA_FUSED_STAGED",
    "GSA_EXPAND_RR",     "GSA_BATCH_ORDER", "GSA_SCORE_SCAN",   "GSA_SCORE_KERNEL",  "GSA_SCORE_K",
    "GSA_SCORE_BIDI",    "GSA_SCORE_BIDI_SW", "GSA_BIDI_GRAN",  "GSA_BIDI_SKEW",     "GSA_BIDI_SW_CONT",
    "GSA_BIDI_LOG",      "GSA_TRACE_BAND",  "GSA_TRACE_BAND_BUDGET", "GSA_STAMPS"};

bool knob_known(const char* name)
{
    for (const char* k : kKnobNames)
        if (std::strcmp(k, name) == 0) return true;
    return false;
}

// the knob's value in this context, or null (unset)
const char* knob(const gsa_ctx* ctx, const char* name)
{
    auto it = ctx->knobs.find(name);
    return it == ctx->knobs.end() ? nullptr : it->second.c_str();
}

int env_int(const gsa_ctx* ctx, const char* name, int dflt)
{
    const char* e = knob(ctx, name);
    return e ? std::atoi(e) : dflt;
}

// Sparse fills run on the K-rows-per-lane kernel (nw_krow.hip, K = 4): 5.9 vs 8.0 ms for the
// 100k pair and 5.7 vs 4.3 TCUPS for 512 pairs of 20k against the strip kernel (nw_strip.hip).
// mlsppt runs on the K-rows kernel too, in its (NS 4, K 4) geometry (one tile row per ticket,
// enqueue_batch).  GSA_SPARSE_KERNEL=strip forces the strip kernel (read per launch, tested);
// GSA_KROW_K (2, 4) and GSA_KROW_NS (2, 4, 8) pick the K-rows geometry.
enum SparseKern { kSpStrip, kSpKrow };
SparseKern sparse_kernel(const gsa_ctx* ctx)
{
    const char* e = knob(ctx, "GSA_SPARSE_KERNEL");
    return (e && std::strcmp(e, "strip") == 0) ? kSpStrip : kSpKrow;
}



// Full fills run on the one-row-per-lane kernel (nw_lane.hip); GSA_LANE_NS = lane strips per
// workgroup (1..4, 6, 8; read per launch, tested; 4 is the default and the fastest measured).
int lane_ns(const gsa_ctx* ctx)
{
    const char* e = knob(ctx, "GSA_LANE_NS");
    const int v = e ? std::atoi(e) : gsa::kLaneNSDefault;
    return ((v >= 1 && v <= 4) || v == 6 || v == 8) ? v : gsa::kLaneNSDefault;
}

// NULL is the HIP null stream, as everywhere in HIP; the host-buffer entry points use the
// context's own stream explicitly.
hipStream_t pick_stream(gsa_ctx*, void* stream) { return (hipStream_t)stream; }

// Device bytes this context holds (scratch, hand-off granules, the host entry points' I/O buffers).
// Units of the *_cap fields: bytes for tmoves, tdirs, tband, dcap, excap and exdesc_cap; ints for
// sbnd, tlist and bidi; 8-byte words for xdone, stamps and clk.
long long held_bytes(const gsa_ctx* c)
{
    long long b = 256 + 64 + (long long)c->gran_elems * 8 + (long long)c->desc_cap * (long long)sizeof(gsa::PairDesc) +
                  (long long)c->tmoves_cap + (long long)c->tdirs_cap + (long long)c->sbnd_cap * 4 +
                  (long long)c->tband_cap + (long long)c->tlist_cap * 4 + (long long)c->excap +
                  (long long)c->exdesc_cap + (long long)c->excap2 + (long long)c->exdesc_cap2 +
                  8 * (long long)(c->xdone_cap + c->stamps_cap + c->clk_cap) +
                  4 * (long long)c->bidi_cap;
    for (size_t k : c->dcap) b += (long long)k;
    return b;
}

// Fold the footprint of the fill just launched (gsa::g_last_foot) into the context's peaks, as
// updateNwAlgPeakMemUsage does per launch (nwalign_shared.cpp:5-25).
void note_launch(gsa_ctx* c)
{
    const gsa::LaunchFoot& f = gsa::g_last_foot;
    c->mem.glmem_peak_allocs = std::max<int64_t>(c->mem.glmem_peak_allocs, held_bytes(c));
    c->mem.shmem_peak_allocs = std::max<int64_t>(c->mem.shmem_peak_allocs, f.lds_per_wg * f.active_wgs);
    c->mem.locmem_peak_allocs =
        std::max<int64_t>(c->mem.locmem_peak_allocs, f.scratch_per_lane * f.threads_per_wg * f.active_wgs);
    c->mem.regmem_peak_allocs =
        std::max<int64_t>(c->mem.regmem_peak_allocs, f.regs_per_lane * 4 * f.threads_per_wg * f.active_wgs);
}

// Read the sticky error word (after the caller's stream sync) and clear it if set.
hipError_t take_err(gsa_ctx* ctx, hipStream_t st, unsigned* err)
{
    hipError_t e = hipMemcpyAsync(err, ctx->ctl + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess && *err != 0)
    {
        e = hipMemsetAsync(ctx->ctl + 1, 0, sizeof(unsigned), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    return e;
}

// Verification launch (nw_check.hip): zero the result words, launch, read them back.
int run_check(gsa_ctx* ctx, gsa::CheckArgs& a, bool sparse, hipStream_t st, gsa_check_result* out)
{
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (!ctx->chk && (e = hipMalloc(&ctx->chk, 64)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    const unsigned long long init[3] = {0ull, 0ull, ~0ull};
    unsigned long long res[3];
    if ((e = hipMemcpyAsync(ctx->chk, init, sizeof(init), hipMemcpyHostToDevice, st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    a.res = ctx->chk;
    e = sparse ? gsa::launch_check_sparse(a, ctx->cu_count, st) : gsa::launch_check_full(a, st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    if ((e = hipMemcpyAsync(res, ctx->chk, sizeof(res), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    out->checked = (int64_t)res[0];
    out->mismatches = (int64_t)res[1];
    out->first = res[1] ? (int64_t)res[2] : -1;
    return GSA_SUCCESS;
}

// Score-only kernels: global alignments run on the strip kernel in its affine mode (shifted
// Gotoh, nw_strip.hip kModeScoreAG); local ones on the row scan (nw_scan.hip).  GSA_SCORE_SCAN=1
// sends global ones to the row scan as well (tests compare the two).
bool score_scan_forced(const gsa_ctx* ctx)
{
    const char* e = knob(ctx, "GSA_SCORE_SCAN");
    return e && std::atoi(e) == 1;
}

constexpr int kScoreTooLarge = 1000;  // internal: score_ag_strip -> row scan

// score-only fills on the K-rows layout (default) or, with GSA_SCORE_KERNEL=strip, the strip kernel
bool score_kernel_krow(const gsa_ctx* ctx)
{
    const char* e = knob(ctx, "GSA_SCORE_KERNEL");
    return !(e && std::strcmp(e, "strip") == 0);
}

// SW end-cell keys: score << bits | (2^bits-1 - row-major index), bits = ceil(log2((R+1)(C+1)));
// scores (< 2^31) keep 63 - bits >= 29 bits up to (R+1)(C+1) = 2^34
int sw_idx_bits(int64_t R, int64_t C)
{
    const unsigned long long n = (unsigned long long)(R + 1) * (unsigned long long)(C + 1) - 1;
    return n ? 64 - __builtin_clzll(n) : 1;
}

// Score-only NW from both ends (nw_bidi.h): a single pair's wavefront time is (C + strips x hop)
// steps, and at 50k the strips' fill-in is ~30 % of it; the top half (rows 1..m) forward and the
// bottom half reversed (rows R..m+1 of the reversed pair) run at the same time, each with half the
// strips, as two pairs of one launch with their tickets interleaved, and a combine kernel takes the
// best crossing of the rows where they meet.  m = K floor(R/2K), so that row m of the top and row
// R - m of the reversed bottom are both a lane's last row (the strips' tap); R % K != 0 takes the
// one-direction path.
// Local modes (SW) run three pairs: the top half forward, the bottom half reversed, and the bottom
// half forward from a fresh (zero) border, whose end-cell keys (offset by m rows) share the top's
// swBest.  The keys then hold the best cell of every alignment that does not cross row m, first in
// row-major order, and the combine the best score through row m (M_cross).  If M_cross is below
// that score, or equal to it with the key's cell in the top half (before every crossing end), the
// key is the answer; otherwise an alignment through row m may end earlier or score more: when the top
// half ended on a ticket boundary, a second launch continues the pair from its ticket there, its row
// above the top's last-ticket granules (restamped), and the answer is the better of the top's keys
// and that run's (GSA_BIDI_SW_CONT=0: not); else the caller runs the one-direction kernel
// (kBidiFallback).
constexpr int kScoreTooLargeB = -1001;
constexpr int kBidiFallback = -1002;
int score_bidi(gsa_ctx* ctx, const int32_t* seqY, int64_t R, const int32_t* seqX, int64_t C, const int32_t* subst,
               int32_t substsz, int32_t gapo, int32_t gape, int K, bool transposed, gsa_score_result* out,
               hipStream_t st, bool local = false)
{
    const int64_t TR = (int64_t)(64 * K) * gsa::kSparseNS;
    const bool affine = gapo != gape;
    // The split.  A half whose rows end on a ticket boundary needs no lane tap: its last ticket's
    // drain writes that row to the granules like any other ticket's, and the combine reads it there.
    // A lane tap costs its strip 8 global stores per block, and as the half's last strip it sets the
    // half's end (50k NW-AG 2.94 ms with no tap, 3.19 with two lane taps).  So the top half ends on a
    // ticket boundary and takes the rows that make both halves end together: skew = p C 64K / (2 hop)
    // rows past R/2, p the lane tap's share of the C steps (0.117 affine, 0.05 linear: 8 / 4 stores
    // per block) and hop ~96 steps between strips; the bottom, when R is a multiple of the ticket too,
    // is free as well and the split even.  Short pairs keep two lane taps (m = K floor(R/2K)).
    int64_t m = (int64_t)K * (R / (2 * K));
    bool topFree = false, botFree = false;
    if (R >= 4 * TR && env_int(ctx, "GSA_BIDI_GRAN", 1))
    {
        const int skewEnv = env_int(ctx, "GSA_BIDI_SKEW", -1);
        // (local linear: 0.075, the third pair's share of the chip moves the balance; 50k SW-LG
        // 2.78 -> 2.76 ms, profiles/r05_sw_skew.txt)
        const double p = affine ? 0.117 : local ? 0.075 : 0.05;
        const bool both = R % TR == 0;
        const int64_t skew = both ? 0 : skewEnv >= 0 ? skewEnv : (int64_t)(p * (double)C * 64.0 * K / (2.0 * 96.0));
        int64_t mt = TR * (int64_t)llround((double)(R / 2 + skew) / (double)TR);
        mt = std::min(std::max(mt, TR), (R - 2 * K) / TR * TR);
        if (mt >= TR && R - mt >= 2 * K && (R - mt) % K == 0)
        {
            m = mt;
            topFree = true;
            botFree = both;
        }
    }
    const int64_t mb = R - m;
    const int64_t tkTop = (m + TR - 1) / TR, tkBot = (mb + TR - 1) / TR;
    const int nP = local ? 3 : 2;
    const size_t tapLen = ((size_t)gsa::kTapPad + (size_t)C + 160 + 63) & ~(size_t)63;
    // layout (ints): tap rows H, F of the top, then of the bottom; reversed Y (mb + 1), reversed X
    // (C + 1), the combine's result
    const size_t oRY = 4 * tapLen, oRX = oRY + (size_t)mb + 1, oRes = (oRX + (size_t)C + 1 + 63) & ~(size_t)63;
    const size_t oSub = oRes + 64;  // transposed: the table transposed
    const size_t need = oSub + (size_t)substsz * (size_t)substsz;
    hipError_t e;
    if (ctx->bidi_cap < need || !ctx->bidi)
    {
        if (ctx->bidi) (void)hipFree(ctx->bidi);
        ctx->bidi = nullptr;
        ctx->bidi_cap = 0;
        if ((e = hipMalloc(&ctx->bidi, need * sizeof(int))) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        ctx->bidi_cap = need;
    }
    if (!ctx->sctl && (e = hipMalloc(&ctx->sctl, 64)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    int* tapH = ctx->bidi;
    int* tapF = tapH + tapLen;  // half 1: + 2 tapLen
    int* ry = ctx->bidi + oRY;
    int* rx = ctx->bidi + oRX;
    int* res = ctx->bidi + oRes;
    int* substT = transposed ? ctx->bidi + oSub : nullptr;
    int s = ensure_desc(ctx, local ? 4 : 2);
    if (s != GSA_SUCCESS) return s;
    const size_t stride = (size_t)gsa::gran_stride((int)C);
    const size_t granAll = (size_t)(tkTop + (nP - 1) * tkBot) * stride;
    const int64_t tkAll = (R + TR - 1) / TR;  // local, the way back: the whole pair's tickets
    if ((s = ensure_gran(ctx, 2 * granAll + (local ? 2 * (size_t)tkAll * stride : 0), st)) != GSA_SUCCESS) return s;
    gsa::PairDesc d[3];
    std::memset(d, 0, sizeof(d));
    d[0].seqY = seqY;
    d[0].seqX = seqX;
    d[0].R = (int)m;
    d[0].nTickets = (int)tkTop;
    d[0].granOff = 0;
    d[1].seqY = ry;
    d[1].seqX = rx;
    d[1].R = (int)mb;
    d[1].nTickets = (int)tkBot;
    d[1].granOff = (long long)((size_t)tkTop * stride);
    // local: the bottom half forward, rows m+1 .. R (seqY + m: its element 0 is row m's letter,
    // unused), from a fresh border
    d[2].seqY = seqY + m;
    d[2].seqX = seqX;
    d[2].R = (int)mb;
    d[2].nTickets = (int)tkBot;
    d[2].granOff = (long long)((size_t)(tkTop + tkBot) * stride);
    d[2].rowOff = (int)m;
    // local: keys of the top (StripArgs::swBest, word 1), of the reversed bottom (word 4, unused) and
    // of the fresh bottom (word 5)
    if (local)
    {
        d[1].swBest = ctx->sctl + 4;
        d[2].swBest = ctx->sctl + 5;
    }
    for (int h = 0; h < 3; ++h) d[h].C = d[h].Cp = (int)C;
    const int mode = local ? (affine ? gsa::kModeScoreSW : gsa::kModeScoreSWL) : affine ? gsa::kModeScoreAG : gsa::kModeScoreAGL;
    const int q8env = env_int(ctx, "GSA_KROW_Q8", 1);
    const int q8 =
        (q8env != 0 && (q8env == 2 || K == 4) && gsa::krow_score_lds_bytes(substsz, true) <= (size_t)ctx->lds_max) ? 1 : 0;
    gsa::StripArgs a;
    std::memset(&a, 0, sizeof(a));
    a.subst = transposed ? substT : subst;
    a.substsz = substsz;
    a.g = gapo;
    a.go = gapo;
    a.ge = gape;
    a.ns = gsa::kSparseNS;
    a.pairs = ctx->desc;
    a.nPairs = nP;
    a.nTicketsTotal = (int)(tkTop + (nP - 1) * tkBot);
    a.bidiTop = (int)tkTop;
    a.bidiMid = local ? (int)tkBot : 0;
    a.gran = ctx->gran;
    a.gran2 = ctx->gran + granAll;
    a.ticket = ctx->ctl;
    a.q8flag = ctx->ctl + 2;
    a.err = (unsigned*)(ctx->sctl + 3);
    a.agResult = (int*)ctx->sctl;
    a.swBest = ctx->sctl + 1;
    a.spin = ctx->spin_ticks;
    a.idxBits = sw_idx_bits(R, C);
    a.epoch = ++ctx->epoch;
    if (a.epoch == 0) a.epoch = ++ctx->epoch;
    a.q8 = q8;
    a.tapRow = topFree ? 0 : (int)m;
    a.tapRowB = botFree ? 0 : (int)mb;
    a.tapGran = (topFree ? 1 : 0) | (botFree ? 2 : 0);
    a.tapH = tapH;
    a.tapF = tapF;
    a.tapStride = (int)(2 * tapLen);
    (void)hipEventRecord(ctx->ev0, st);
    if ((e = gsa::launch_bidi_prep(d[0], d[1], ctx->desc, seqY, (int)m, (int)R, seqX, (int)C, ry, rx, ctx->ctl, ctx->sctl,
                                   res, subst, substsz, substT, st, local ? &d[2] : nullptr)) != hipSuccess ||
        (e = gsa::launch_krow_score(a, mode, K, std::max(1, std::min(a.nTicketsTotal, ctx->cu_count)), st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    note_launch(ctx);
    // the rows where the halves meet: a lane tap (tap rows, one int per column from kTapPad), or the
    // half's last-ticket granules (the low word of each 64-bit granule)
    const int* gTop = (const int*)(ctx->gran + (size_t)(tkTop - 1) * stride);
    const int* gBot = (const int*)(ctx->gran + (size_t)(tkTop + tkBot - 1) * stride);
    const int* tH = topFree ? gTop : tapH + gsa::kTapPad;
    const int* tF = topFree ? gTop + 2 * granAll : tapF + gsa::kTapPad;
    const int* bH = botFree ? gBot : tapH + 2 * tapLen + gsa::kTapPad;
    const int* bF = botFree ? gBot + 2 * granAll : tapF + 2 * tapLen + gsa::kTapPad;
    if ((e = gsa::launch_bidi_combine(tH, tF, topFree ? 2 : 1, bH, bF, botFree ? 2 : 1, (int)m, (int)mb, (int)C, gapo,
                                      gape, affine, res, st, local)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    (void)hipEventRecord(ctx->ev1, st);
    unsigned long long rw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int score = 0;
    if ((e = hipMemcpyAsync(rw, ctx->sctl, sizeof(rw), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemcpyAsync(&score, res, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    (void)hipEventElapsedTime(&out->calc_kernel_ms, ctx->ev0, ctx->ev1);
    const unsigned err = (unsigned)rw[3];
    if (err == 2u) return kScoreTooLargeB;  // a value outside int16: the row scan
    if (err != 0) return GSA_ERROR_KERNEL_FAILURE;
    if (local)
    {
        if (rw[0] & 1u) return kScoreTooLargeB;  // a score >= 2^26: the row scan
        const int bits = sw_idx_bits(R, C);
        const unsigned long long mask = (1ull << bits) - 1;
        unsigned long long key = std::max(rw[1], rw[5]);  // top, fresh bottom
        unsigned long long idx = key ? mask - (key & mask) : 0;
        long long best = key ? (long long)(key >> bits) : 0;
        const long long ie = (long long)(idx / (unsigned long long)(C + 1));
        const bool fallback = !((long long)score < best || ((long long)score == best && ie <= m));
        const bool cont = fallback && topFree && env_int(ctx, "GSA_BIDI_SW_CONT", 1) != 0;
        if (env_int(ctx, "GSA_BIDI_LOG", 0))  // (tests: which way the pair went)
            std::fprintf(stderr, "gsa local both ends: m %lld, through m %d, best off it %lld at row %lld -> %s\n",
                         (long long)m, score, best, ie,
                         !fallback ? "answer" : cont ? "bottom again from row m" : "one direction");
        if (fallback && !cont) return kBidiFallback;
        if (cont)
        {
            // the pair from ticket tkTop on, its row above the top's last-ticket granules, in a granule
            // area of its own (its later tickets must not meet another half's granules)
            unsigned long long* seedH = ctx->gran + 2 * granAll;
            unsigned long long* seedF = seedH + (size_t)tkAll * stride;
            unsigned ep2 = ++ctx->epoch;
            if (ep2 == 0) ep2 = ++ctx->epoch;
            const size_t last = (size_t)(tkTop - 1) * stride;
            gsa::PairDesc dc;
            std::memset(&dc, 0, sizeof(dc));
            dc.seqY = seqY;
            dc.seqX = seqX;
            dc.R = (int)R;
            dc.C = dc.Cp = (int)C;
            dc.nTickets = (int)tkAll;
            dc.swBest = ctx->sctl + 6;
            gsa::StripArgs b = a;
            b.pairs = ctx->desc + 3;
            b.nPairs = 1;
            b.bidiTop = b.bidiMid = 0;
            b.nTicketsTotal = (int)(tkAll - tkTop);
            b.tkFirst = (int)tkTop;
            b.gran = seedH;
            b.gran2 = seedF;
            b.epoch = ep2;
            b.tapRow = b.tapRowB = b.tapGran = 0;
            if ((e = hipMemcpyAsync(ctx->desc + 3, &dc, sizeof(dc), hipMemcpyHostToDevice, st)) != hipSuccess ||
                (e = hipMemsetAsync(ctx->ctl, 0, 4, st)) != hipSuccess ||
                (e = hipMemsetAsync(ctx->sctl, 0, 8, st)) != hipSuccess ||
                (e = hipMemsetAsync(ctx->sctl + 6, 0, 8, st)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
            if ((e = gsa::launch_bidi_seed(ctx->gran + last, affine ? ctx->gran + granAll + last : nullptr, seedH + last,
                                           affine ? seedF + last : nullptr, (long long)stride, ep2, st)) != hipSuccess ||
                (e = gsa::launch_krow_score(b, mode, K, std::max(1, std::min(b.nTicketsTotal, ctx->cu_count)), st)) !=
                    hipSuccess)
                return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
            note_launch(ctx);
            (void)hipEventRecord(ctx->ev1, st);
            if ((e = hipMemcpyAsync(rw, ctx->sctl, sizeof(rw), hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipStreamSynchronize(st)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
            (void)hipEventElapsedTime(&out->calc_kernel_ms, ctx->ev0, ctx->ev1);
            const unsigned err2 = (unsigned)rw[3];
            if (err2 == 2u) return kScoreTooLargeB;
            if (err2 != 0) return GSA_ERROR_KERNEL_FAILURE;
            if (rw[0] & 1u) return kScoreTooLargeB;
            key = std::max(rw[1], rw[6]);  // the top's keys (word 1 is not touched again), the rest's
            idx = key ? mask - (key & mask) : 0;
            best = key ? (long long)(key >> bits) : 0;
        }
        out->score = (int32_t)best;
        out->i_end = (int64_t)(idx / (unsigned long long)(C + 1));
        out->j_end = (int64_t)(idx % (unsigned long long)(C + 1));
        return GSA_SUCCESS;
    }
    out->score = score;
    out->i_end = transposed ? C : R;
    out->j_end = transposed ? R : C;
    return GSA_SUCCESS;
}

int score_ag_strip(gsa_ctx* ctx, const int32_t* seqY, int64_t R, const int32_t* seqX, int64_t C, const int32_t* subst,
                   int32_t substsz, int32_t gapo, int32_t gape, int32_t local, gsa_score_result* out, hipStream_t st)
{
    // the K-rows score kernel's rows per lane, tickets of 64 K NS rows: 2 in the modes with the
    // longer step (SW tracking, affine gaps: the block's fixed part is a smaller share there, and
    // twice the strips shorten it), 4 for NW-LG; same box, 5k-100k pairs: NW-AG -5..-7 %, SW-AG
    // -9..-11 %, SW-LG -2..-5 % with 2, NW-LG +12..18 % (profiles/r04_score_k.txt).  GSA_SCORE_K
    // = 2 / 4 forces one
    const int kenv = env_int(ctx, "GSA_SCORE_K", 0);
    const int scoreK = kenv == 2 || kenv == 4 ? kenv : (!local && gapo == gape) ? 4 : 2;
    // the K-rows score kernel unless GSA_SCORE_KERNEL=strip, or its LDS (a profile of substsz rows)
    // does not fit, or SW with ge > 0 (its per-row key offsets assume z grows along j); the strip
    // kernel's score modes otherwise, on its own 1024-row tickets
    const bool krow = score_kernel_krow(ctx) && (!local || gape <= 0) && gsa::krow_score_lds_bytes(substsz) <= ctx->lds_max;
    const int64_t TR = krow ? (int64_t)(64 * scoreK) * gsa::kSparseNS : (int64_t)gsa::kWaveRows * gsa::kSparseNS;
    const int64_t tickets = (R + TR - 1) / TR;
    if (tickets > (1ll << 30) || C > (1ll << 30)) return GSA_ERROR_INVALID_VALUE;
    // NW from both ends (score_bidi) when each half keeps >= 4 tickets, at 2 rows per lane in both
    // NW modes (its halves have half the strips, so the shorter block wins for NW-LG too: 50k 2.25 ->
    // 2.11 ms, profiles/r05_bidi_ab.txt).  GSA_SCORE_BIDI: 0 never, 2 at any size (tests)
    // A pair whose R is not a multiple of K but whose C is runs transposed (X down the rows, Y along
    // them, the table transposed: the same global score, and gaps cost the same either way).
    const int bidi = env_int(ctx, "GSA_SCORE_BIDI", 1);
    const int kb = kenv == 2 || kenv == 4 ? kenv : 2;
    const int64_t TRb = (int64_t)(64 * kb) * gsa::kSparseNS;
    auto splits = [&](int64_t rows) { return rows % kb == 0 && rows >= 2 * kb && (bidi == 2 || rows >= 8 * TRb); };
    if (krow && !local && bidi != 0 && (splits(R) || splits(C)))
    {
        const bool tr = !splits(R);
        const int sb = tr ? score_bidi(ctx, seqX, C, seqY, R, subst, substsz, gapo, gape, kb, true, out, st)
                          : score_bidi(ctx, seqY, R, seqX, C, subst, substsz, gapo, gape, kb, false, out, st);
        return sb == kScoreTooLargeB ? kScoreTooLarge : sb;
    }
    // local: from both ends only by rows (the end cell's row-major tie rule does not survive a
    // transpose), and back to one direction when an alignment through the split may decide it
    float bidiMs = 0.f;
    if (krow && local && bidi != 0 && env_int(ctx, "GSA_SCORE_BIDI_SW", 1) && splits(R))
    {
        const int sb = score_bidi(ctx, seqY, R, seqX, C, subst, substsz, gapo, gape, kb, false, out, st, true);
        if (sb == kScoreTooLargeB) return kScoreTooLarge;
        if (sb != kBidiFallback) return sb;
        bidiMs = out->calc_kernel_ms;
    }
    gsa::StripArgs a;
    std::memset(&a, 0, sizeof(a));
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    a.go = gapo;
    a.ge = gape;
    a.ns = gsa::kSparseNS;
    gsa::PairDesc d;
    std::memset(&d, 0, sizeof(d));
    d.seqY = seqY;
    d.seqX = seqX;
    d.R = (int)R;
    d.C = (int)C;
    d.Cp = (int)C;
    d.nTickets = (int)tickets;
    int s = ensure_desc(ctx, 1);
    if (s != GSA_SUCCESS) return s;
    hipError_t e = hipMemcpyAsync(ctx->desc, &d, sizeof(d), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    const size_t gran = (size_t)tickets * (size_t)gsa::gran_stride((int)C);
    if ((s = ensure_gran(ctx, 2 * gran, st)) != GSA_SUCCESS) return s;
    if (!ctx->sctl && (e = hipMalloc(&ctx->sctl, 64)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    a.pairs = ctx->desc;
    a.nPairs = 1;
    a.nTicketsTotal = (int)tickets;
    a.gran = ctx->gran;
    a.gran2 = ctx->gran + gran;
    a.ticket = ctx->ctl;
    // an error word of its own: a fill enqueued earlier on this stream keeps its sticky error for
    // the caller's gsa_sync, and its error does not read as this launch's
    a.err = (unsigned*)(ctx->sctl + 3);
    a.spin = ctx->spin_ticks;
    a.agResult = (int*)ctx->sctl;
    a.swBest = ctx->sctl + 1;
    a.idxBits = sw_idx_bits(R, C);
    a.epoch = ++ctx->epoch;
    if (a.epoch == 0) a.epoch = ++ctx->epoch;
    if ((e = hipMemsetAsync(ctx->ctl, 0, 4, st)) != hipSuccess || (e = hipMemsetAsync(ctx->sctl, 0, 32, st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    (void)hipEventRecord(ctx->ev0, st);
    const int grid = std::max(1, std::min((int)tickets, ctx->cu_count));
    // a linear gap (gapo == gape) runs the step without E' and F' (d = 0)
    const int mode = local ? (gapo == gape ? gsa::kModeScoreSWL : gsa::kModeScoreSW)
                           : (gapo == gape ? gsa::kModeScoreAGL : gsa::kModeScoreAG);
    // the int8 column profile where its LDS fits (the instance declines a table outside int8 and the
    // int16 instance behind it runs) for the 4-rows-per-lane geometry (NW-LG): 50k 2.52 -> 2.46 ms;
    // at 2 rows per lane the int16 profile is faster (SW-LG 3.71 -> 3.42 ms, NW-AG 4.16 -> 3.87;
    // profiles/r04_score_k.txt).  GSA_KROW_Q8=0 / 2: int16 / int8 always
    const int q8env = env_int(ctx, "GSA_KROW_Q8", 1);
    a.q8 = (q8env != 0 && (q8env == 2 || scoreK == 4) && gsa::krow_score_lds_bytes(substsz, true) <= (size_t)ctx->lds_max) ? 1 : 0;
    a.q8flag = ctx->ctl + 2;
    if ((e = krow ? gsa::launch_krow_score(a, mode, scoreK, grid, st) : gsa::launch_strip_fill(a, mode, grid, st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    note_launch(ctx);
    (void)hipEventRecord(ctx->ev1, st);
    unsigned long long res[4] = {0, 0, 0, 0};
    if ((e = hipMemcpyAsync(res, ctx->sctl, sizeof(res), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    const unsigned err = (unsigned)res[3];
    (void)hipEventElapsedTime(&out->calc_kernel_ms, ctx->ev0, ctx->ev1);
    out->calc_kernel_ms += bidiMs;  // (a local pair back from both ends: both launches)
    // a substitution value outside int16 after the shift: the int32 row scan computes it
    if (err == 2u) return kScoreTooLarge;
    if (err != 0) return GSA_ERROR_KERNEL_FAILURE;
    if (local)
    {
        if (res[0] & 1u) return kScoreTooLarge;  // a score >= 2^26: the caller takes the row scan
        // max key: score << idxBits | (2^idxBits-1 - row-major index); 0 = no positive cell -> (0, 0, 0)
        const int bits = sw_idx_bits(R, C);
        const unsigned long long mask = (1ull << bits) - 1;
        const unsigned long long idx = res[1] ? mask - (res[1] & mask) : 0;
        out->score = (int32_t)(res[1] >> bits);
        out->i_end = (int64_t)(idx / (unsigned long long)(C + 1));
        out->j_end = (int64_t)(idx % (unsigned long long)(C + 1));
        return GSA_SUCCESS;
    }
    out->score = (int32_t)(uint32_t)res[0];
    out->i_end = R;
    out->j_end = C;
    return GSA_SUCCESS;
}

// The fused two-pass full fill's launch (enqueue_full_twopass): the expansion's arguments, the
// pass-1 geometry (ns strips per ticket), the workgroup's waves and the workgroups that take pass-1
// tickets first
struct FusedLaunch
{
    const gsa::ExpandArgs* xa;
    int ns, waves, p1;
    bool staged;  // nw_full_fused_kernel's row-64m hand-off through a storer wave (PTF 3), else direct
};

// One batched launch: headers of every pair, then the persistent strip kernel over the
// tickets of all pairs (pair-major).  `pairs` holds device pointers.
int enqueue_batch(gsa_ctx* ctx, int mode, int npairs, const gsa_pair_dev* pairs, const int32_t* subst, int32_t substsz,
                  int32_t gapo, int32_t tileBx, hipStream_t st, unsigned long long* done = nullptr, int ptChunk = 0,
                  const int32_t* lds = nullptr, int* const* rows64 = nullptr, const FusedLaunch* fused = nullptr)
{
    if (npairs < 1 || !pairs || !subst) return GSA_ERROR_INVALID_VALUE;
    if (substsz < 1 || substsz > 32) return GSA_ERROR_INVALID_VALUE;  // LDS profile holds <= 32 letters
    gsa::StripArgs a;
    std::memset(&a, 0, sizeof(a));
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    const bool lane = mode == gsa::kModeFull;
    // mlsppt publishes column chunks from the K-rows kernel only
    const bool krow = mode == gsa::kModeSparse && (sparse_kernel(ctx) == kSpKrow || done || rows64);
    // single pairs: 4 strips per workgroup (each on its own SIMD: the pair's critical path);
    // batches: 8 (two strips per SIMD share the issue slots a single strip leaves idle, 512 x 20k
    // 5.7 -> 7.3 TCUPS; a single 100k pair 5.9 -> 8.4 ms), unless the batch's 4-strip tickets
    // (one tile row each) all fit the chip at once: then every pair runs on its critical path
    long long tileRows = 0;
    for (int p = 0; p < npairs; ++p)
        tileRows += std::max<long long>(1, ((long long)pairs[p].adjrows - 1 + gsa::kSparseTileBy - 1) / gsa::kSparseTileBy);
    const bool fitsChip = tileRows <= (long long)std::max(1, ctx->cu_count);
    const int nsDefault = (npairs > 1 && !fitsChip) ? gsa::kKrowNSBatchDefault : gsa::kKrowNSDefault;
    int krowK = env_int(ctx, "GSA_KROW_K", gsa::kKrowKDefault), krowNS = env_int(ctx, "GSA_KROW_NS", nsDefault);
    if (rows64)  // pass 1 of the two-pass full fill: the XR instances, K = 4 on 4 or 8 strips
    {
        krowK = 4;
        krowNS = fused ? fused->ns : env_int(ctx, "GSA_KROW_NS", (npairs > 1 && !fitsChip) ? 8 : 4) == 8 ? 8 : 4;
    }
    // mlsppt flags one ticket per tile row: only the geometry whose ticket is one tile row
    if (!gsa::krow_ok(krowNS, krowK) || (done && gsa::krow_ticket_rows(krowNS, krowK) != gsa::kSparseTileBy))
    {
        krowK = gsa::kKrowKDefault;
        krowNS = gsa::kKrowNSDefault;
    }
    a.ns = lane ? lane_ns(ctx) : krow ? krowNS : gsa::kSparseNS;
    // the K-rows fill's int8 column profile (its instance declines a table outside int8 and the int16
    // one runs instead) wherever its LDS fits; GSA_KROW_Q8=0 keeps the int16 profile
    if (krow && env_int(ctx, "GSA_KROW_Q8", 1) != 0)
        a.q8 = gsa::krow_lds_bytes(krowNS, krowNS == 2 ? 512 : 1024, substsz, true) <= (size_t)ctx->lds_max ? 1 : 0;
    a.q8flag = ctx->ctl + 2;
    const int fullRows = gsa::kLaneRows * a.ns;  // rows per ticket of a full fill
    if (mode == gsa::kModeSparse)
    {
        if (tileBx < 64 || tileBx % 16 != 0) return GSA_ERROR_INVALID_VALUE;
        a.tBx = tileBx;
        a.tBy = gsa::kSparseTileBy;
    }
    std::vector<gsa::PairDesc> hd((size_t)npairs);
    long long tickets = 0, gran = 0, maxWork = 1;
    for (int p = 0; p < npairs; ++p)
    {
        const gsa_pair_dev& in = pairs[p];
        if (in.adjrows < 1 || in.adjcols < 1 || !in.seqY || !in.seqX) return GSA_ERROR_INVALID_VALUE;
        gsa::PairDesc& d = hd[(size_t)p];
        std::memset(&d, 0, sizeof(d));
        d.seqY = in.seqY;
        d.seqX = in.seqX;
        d.R = in.adjrows - 1;
        d.C = in.adjcols - 1;
        if (mode == gsa::kModeFull)
        {
            if (!in.score) return GSA_ERROR_INVALID_VALUE;
            d.score = in.score;
            // row pitch: unpadded, or the caller's (gsa_full_pitch gives the one whose anti-diagonals
            // share their 128-byte line offset, so the strips' row segments are whole lines)
            d.ld = lds ? lds[p] : in.adjcols;
            if (d.ld < in.adjcols) return GSA_ERROR_INVALID_VALUE;
            d.Cp = d.C;
            // an empty row or column leaves nothing but headers to compute
            d.nTickets = (d.C == 0) ? 0 : (d.R + fullRows - 1) / fullRows;
            maxWork = std::max<long long>(maxWork, (long long)std::max(d.R, d.C) + 1);
        }
        else
        {
            if (!in.tileHrowMat || !in.tileHcolMat) return GSA_ERROR_INVALID_VALUE;
            gsa_sparse_geom geom;
            int s = gsa_sparse_geometry(in.adjrows, in.adjcols, tileBx, &geom);
            if (s != GSA_SUCCESS) return s;
            d.hrow = in.tileHrowMat;
            d.hcol = in.tileHcolMat;
            d.trows = geom.tileHdrMatRows;
            d.tcols = geom.tileHdrMatCols;
            d.Cp = d.tcols * tileBx;
            d.nTickets = krow ? gsa::krow_tickets(d.trows, krowNS, krowK) : d.trows;
            if (rows64)
            {
                d.rows64 = rows64[p];
                d.rpitch = gsa::rows64_pitch(d.Cp);
            }
            maxWork = std::max<long long>(maxWork, std::max((long long)d.tcols * (tileBx + 1),
                                                            (long long)d.trows * (gsa::kSparseTileBy + 1)));
        }
        d.ticketBase = (int)tickets;
        d.granOff = gran;
        tickets += d.nTickets;
        gran += (long long)d.nTickets * gsa::gran_stride(d.Cp);
        if (tickets > (1ll << 30)) return GSA_ERROR_INVALID_VALUE;
    }
    // batch schedule (more than one pair): round-robin over the pairs, longest first, so the
    // resident workgroups run the first tickets of every pair side by side instead of one pair's
    // chain of dependent tickets; ticket j of a pair stays behind its ticket j-1
    std::vector<int> sched;
    const char* order = knob(ctx, "GSA_BATCH_ORDER");  // "pair": pair-major (comparisons)
    if (npairs > 1 && !(order && std::strcmp(order, "pair") == 0))
    {
        std::vector<int> ord((size_t)npairs);
        for (int p = 0; p < npairs; ++p) ord[(size_t)p] = p;
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return hd[(size_t)x].nTickets > hd[(size_t)y].nTickets; });
        sched.reserve(2 * (size_t)tickets);
        for (int j = 0; j < hd[(size_t)ord[0]].nTickets; ++j)
            for (int p : ord)
            {
                if (hd[(size_t)p].nTickets <= j) break;
                sched.push_back(p);
                sched.push_back(j);
            }
    }
    // descriptors, then the schedule, in one device buffer (units of PairDesc)
    const size_t schedUnits = (sched.size() * sizeof(int) + sizeof(gsa::PairDesc) - 1) / sizeof(gsa::PairDesc);
    const size_t units = (size_t)npairs + schedUnits;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    int s = ensure_desc(ctx, units);
    if (s != GSA_SUCCESS) return s;
    // stage the descriptors in a pinned slot and copy them in stream order
    const int slot = ctx->stage_next;
    ctx->stage_next = (slot + 1) % gsa_ctx::kStage;
    if (ctx->stage_used[slot] && (e = hipEventSynchronize(ctx->stage_ev[slot])) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (ctx->stage_cap[slot] < units)
    {
        if (ctx->stage[slot]) (void)hipHostFree(ctx->stage[slot]);
        ctx->stage[slot] = nullptr;
        ctx->stage_cap[slot] = 0;
        if ((e = hipHostMalloc((void**)&ctx->stage[slot], units * sizeof(gsa::PairDesc))) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        ctx->stage_cap[slot] = units;
    }
    std::memcpy(ctx->stage[slot], hd.data(), (size_t)npairs * sizeof(gsa::PairDesc));
    if (!sched.empty()) std::memcpy(ctx->stage[slot] + npairs, sched.data(), sched.size() * sizeof(int));
    e = hipMemcpyAsync(ctx->desc, ctx->stage[slot], units * sizeof(gsa::PairDesc), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(ctx->stage_ev[slot], st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    ctx->stage_used[slot] = true;

    a.pairs = ctx->desc;
    a.nPairs = npairs;
    a.nTicketsTotal = (int)tickets;
    a.sched = sched.empty() ? nullptr : (const int*)(ctx->desc + npairs);
    e = gsa::launch_headers(a, mode, maxWork, st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    if (tickets == 0) return GSA_SUCCESS;

    // granule stride (Cp+1) and base are per pair: the kernel takes them from the descriptor
    if ((s = ensure_gran(ctx, (size_t)gran, st)) != GSA_SUCCESS) return s;
    a.gran = ctx->gran;
    a.ticket = ctx->ctl;
    a.err = ctx->ctl + 1;
    a.spin = ctx->spin_ticks;
    a.done = done;
    a.ptChunk = std::max(1, ptChunk);
    a.epoch = ++ctx->epoch;
    if (a.epoch == 0) a.epoch = ++ctx->epoch;  // 0 is the cleared-tag value
    if (fused)
    {
        if (!rows64) return GSA_ERROR_INVALID_VALUE;
        const size_t words = (size_t)tickets * (size_t)krowNS;
        if (ctx->xdone_cap < words || !ctx->xdone)
        {
            if (ctx->xdone) (void)hipFree(ctx->xdone);
            ctx->xdone = nullptr;
            ctx->xdone_cap = 0;
            const size_t cap = std::max<size_t>(words, 1024);
            if ((e = hipMalloc(&ctx->xdone, cap * sizeof(unsigned long long))) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
            if ((e = hipMemsetAsync(ctx->xdone, 0, cap * sizeof(unsigned long long), st)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
            ctx->xdone_cap = cap;
        }
        {
            a.xpair = fused->xa->pairs;
            a.xsched = fused->xa->sched;
            a.xTasks = fused->xa->nTasks;
            a.xrun = fused->xa->run;
            a.xP = fused->p1;
            a.xrole = ctx->ctl + 4;
            a.xcounter = ctx->ctl + 5;
            if ((e = hipMemsetAsync(a.xrole, 0, 8, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
            ctx->stamps_n = 0;
            if (env_int(ctx, "GSA_STAMPS", 0))
            {
                const size_t n = 4 * words + 3 * (size_t)a.xTasks;
                if (ctx->stamps_cap < n)
                {
                    if (ctx->stamps) (void)hipFree(ctx->stamps);
                    ctx->stamps = nullptr;
                    ctx->stamps_cap = 0;
                    if ((e = hipMalloc(&ctx->stamps, n * sizeof(unsigned long long))) != hipSuccess)
                        return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
                    ctx->stamps_cap = n;
                }
                if ((e = hipMemsetAsync(ctx->stamps, 0, n * sizeof(unsigned long long), st)) != hipSuccess)
                    return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
                a.stamps = ctx->stamps;
                ctx->stamps_n = n;
                ctx->stamps_stream = st;
            }
        }
        a.xdone = ctx->xdone;
    }
    if (!fused && krow && !lane && env_int(ctx, "GSA_STAMPS", 0))
    {
        // the K-rows fill's ledger (nw_krow_kernel): 10 words per strip
        const size_t n = 10 * (size_t)tickets * (size_t)krowNS;
        ctx->stamps_n = 0;
        if (ctx->stamps_cap < n)
        {
            if (ctx->stamps) (void)hipFree(ctx->stamps);
            ctx->stamps = nullptr;
            ctx->stamps_cap = 0;
            if ((e = hipMalloc(&ctx->stamps, n * sizeof(unsigned long long))) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
            ctx->stamps_cap = n;
        }
        if ((e = hipMemsetAsync(ctx->stamps, 0, n * sizeof(unsigned long long), st)) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
        a.stamps = ctx->stamps;
        ctx->stamps_n = n;
        ctx->stamps_stream = st;
    }
    e = hipMemsetAsync(ctx->ctl, 0, 4, st);  // the ticket; the error word stays sticky
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    // one pair: one workgroup per CU (its tickets are a chain); a batch: all resident slots
    int grid = (npairs == 1) ? std::max(1, std::min((int)tickets, ctx->cu_count)) : 0;
    a.laneFeed = knob(ctx, "GSA_LANE_FEED") ? env_int(ctx, "GSA_LANE_FEED", 0) : -1;
    a.lanePair = knob(ctx, "GSA_LANE_PAIR") ? env_int(ctx, "GSA_LANE_PAIR", 0) : -1;
    e = lane     ? gsa::launch_lane_fill(a, a.ns, grid, st)
        : fused  ? gsa::launch_full_fused(a, fused->ns, fused->waves, fused->staged, 0, st)
        : rows64 ? gsa::launch_krow_fill_xr(a, krowNS, grid, st)
        : krow   ? gsa::launch_krow_fill(a, krowNS, krowK, 0, grid, st)
                 : gsa::launch_strip_fill(a, mode, grid, st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    note_launch(ctx);
    return GSA_SUCCESS;
}

int enqueue_fill(gsa_ctx* ctx, int mode, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                 const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score, int32_t tileBx, int32_t* hrow,
                 int32_t* hcol, hipStream_t st, unsigned long long* done = nullptr, int ptChunk = 0,
                 const int32_t* ld = nullptr)
{
    gsa_pair_dev p {seqY, adjrows, seqX, adjcols, score, hrow, hcol};
    return enqueue_batch(ctx, mode, 1, &p, subst, substsz, gapo, tileBx, st, done, ptChunk, ld);
}

// enqueue_full_twopass's answer when its pass-1 scratch (header rows and columns plus every 64th
// row, ~2 % of the matrix) does not fit next to the caller's matrix: enqueue_full then runs the
// one-pass lane fill, which needs no scratch
constexpr int kNoScratch = -1000;

// Full fills in two passes (nw_expand.h): pass 1 = the K-rows sparse fill of every pair with tile
// width kExpTW, which also keeps rows 64m (XR instance), into the context's scratch; pass 2 =
// every 64-row x kExpTW tile of every matrix recomputed from its top row and left column at once.
// lds: row pitches (null: unpadded).
// (enqueue_full_split: slot 1 = the tail group's scratch; afterP1 recorded behind pass 1, beforeP1
// awaited before it; split: the caller records the timing events and no clock stamps are taken;
// rr >= 0: that expansion order, untuned; startEv: recorded on st just before pass 1)
struct TwoPassOpts
{
    int slot = 0;
    hipEvent_t afterP1 = nullptr, beforeP1 = nullptr, timeP1 = nullptr, startEv = nullptr;
    bool split = false;
    int rr = -1;
};
int enqueue_full_twopass(gsa_ctx* ctx, int npairs, const gsa_pair_dev* pairs, const int32_t* lds, const int32_t* subst,
                         int32_t substsz, int32_t gapo, hipStream_t st, const TwoPassOpts& opt = TwoPassOpts())
{
    void*& exbuf = opt.slot ? ctx->exbuf2 : ctx->exbuf;
    size_t& excap = opt.slot ? ctx->excap2 : ctx->excap;
    void*& exdesc = opt.slot ? ctx->exdesc2 : ctx->exdesc;
    size_t& exdesc_cap = opt.slot ? ctx->exdesc_cap2 : ctx->exdesc_cap;
    gsa_ctx::XTune& xt = ctx->xt[opt.slot];
    if (npairs < 1 || !pairs || !subst) return GSA_ERROR_INVALID_VALUE;
    if (substsz < 1 || substsz > 32) return GSA_ERROR_INVALID_VALUE;
    // pass-1 geometry as enqueue_batch derives it for the XR instances
    long long tileRows = 0;
    for (int p = 0; p < npairs; ++p)
        tileRows += std::max<long long>(1, ((long long)pairs[p].adjrows - 1 + gsa::kSparseTileBy - 1) / gsa::kSparseTileBy);
    const bool fitsChip = tileRows <= (long long)std::max(1, ctx->cu_count);
    // both passes in one launch (nw_full_fused_kernel) for single pairs; GSA_FULL_FUSED=0: two launches.
    // (A matrix without interior cells has no pass-1 tickets: the expansion alone writes its headers.)
    const int fusedMode = env_int(ctx, "GSA_FULL_FUSED", 1);
    bool interior = true;
    for (int p = 0; p < npairs; ++p) interior = interior && pairs[p].adjrows > 1 && pairs[p].adjcols > 1;
    // (never inside a split batch: a group of one pair would take the fused branch, which records
    // neither afterP1 nor timeP1, and group B would then start against an unrecorded event)
    const bool fused = interior && !opt.split && npairs == 1 && fusedMode >= 1;
    const int ns = env_int(ctx, "GSA_KROW_NS", (npairs > 1 && !fitsChip) ? 8 : 4) == 8 ? 8 : 4;  // as enqueue_batch
    // pass 2 (fused or its own launch): the streamed expansion, kExpStreamWaves - 1 tile waves per
    // workgroup, tasks of that many 64-row tiles
    const int xWaves = gsa::kExpStreamWaves - 1;
    const int xmt = 1;
    std::vector<gsa_pair_dev> p1((size_t)npairs);
    std::vector<gsa::ExpandPair> ex((size_t)npairs);
    std::vector<size_t> off((size_t)npairs * 3);
    size_t bytes = 0;
    auto take = [&](size_t b) {
        const size_t o = bytes;
        bytes += (b + 255) & ~(size_t)255;
        return o;
    };
    long long tasks = 0, strips = 0;
    for (int p = 0; p < npairs; ++p)
    {
        const gsa_pair_dev& in = pairs[p];
        if (in.adjrows < 1 || in.adjcols < 1 || !in.seqY || !in.seqX || !in.score) return GSA_ERROR_INVALID_VALUE;
        const long long ld = lds ? lds[p] : in.adjcols;
        if (ld < in.adjcols) return GSA_ERROR_INVALID_VALUE;
        gsa_sparse_geom geom;
        int s = gsa_sparse_geometry(in.adjrows, in.adjcols, gsa::kExpHB, &geom);
        if (s != GSA_SUCCESS) return s;
        const int Cp = geom.tileHdrMatCols * gsa::kExpHB;
        const long long tickets = gsa::krow_tickets(geom.tileHdrMatRows, ns, 4);
        const long long nrows = tickets * ns * 4;  // rows 64m written by pass 1, m = 1 .. nrows
        off[3 * p] = take((size_t)geom.hrowElems * 4);
        off[3 * p + 1] = take((size_t)geom.hcolElems * 4);
        off[3 * p + 2] = take((size_t)(nrows * gsa::rows64_pitch(Cp)) * 4);
        gsa::ExpandPair& e = ex[(size_t)p];
        std::memset(&e, 0, sizeof(e));
        e.seqY = in.seqY;
        e.seqX = in.seqX;
        e.R = in.adjrows - 1;
        e.C = in.adjcols - 1;
        e.score = in.score;
        e.ld = ld;
        e.rpitch = gsa::rows64_pitch(Cp);
        e.tcols = geom.tileHdrMatCols;
        // (an empty sequence still has its header row or column: at least one task per dimension)
        e.colTiles = std::max(1, (e.C + gsa::kExpTW - 1) / gsa::kExpTW);
        // a last tile column wider than one pass-1 tile is split at its boundary: the pair's last
        // tiles, which wait for the end of pass 1 in a fused fill, are then at most kExpHB wide
        e.lastSplit = e.C - (e.colTiles - 1) * gsa::kExpTW > gsa::kExpHB ? 1 : 0;
        e.colTiles += e.lastSplit;
        e.rowChunks = std::max(1, (e.R + xWaves * gsa::kExpRows * xmt - 1) / (xWaves * gsa::kExpRows * xmt));
        e.taskBase = (int)tasks;
        tasks += (long long)e.colTiles * e.rowChunks;
        e.p1Strip0 = (int)strips;  // (enqueue_batch's ticketBase x ns: pair-major)
        e.p1Strips = (int)(tickets * ns);
        strips += tickets * ns;
        if (tasks > (1ll << 30) || strips > (1ll << 30)) return GSA_ERROR_INVALID_VALUE;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (excap < bytes || !exbuf)
    {
        if (exbuf) (void)hipFree(exbuf);
        exbuf = nullptr;
        excap = 0;
        if ((e = hipMalloc(&exbuf, std::max<size_t>(bytes, 256))) != hipSuccess)
        {
            (void)hipGetLastError();  // the caller falls back to the one-pass lane fill
            return kNoScratch;
        }
        excap = std::max<size_t>(bytes, 256);
    }
    char* base = (char*)exbuf;
    std::vector<int*> rows((size_t)npairs);
    for (int p = 0; p < npairs; ++p)
    {
        p1[(size_t)p] = pairs[p];
        p1[(size_t)p].score = nullptr;
        p1[(size_t)p].tileHrowMat = (int32_t*)(base + off[3 * p]);
        p1[(size_t)p].tileHcolMat = (int32_t*)(base + off[3 * p + 1]);
        rows[(size_t)p] = (int*)(base + off[3 * p + 2]);
        ex[(size_t)p].rows64 = rows[(size_t)p];
        ex[(size_t)p].hcol = p1[(size_t)p].tileHcolMat;
    }
    // the expansion's descriptors and (batches) its round-robin schedule, staged in a pinned slot and
    // copied in stream order
    // Task order of a batch's expansion.  Round-robin over the pairs (one task of every pair in turn)
    // keeps the tasks in flight spread over all matrices, and its pass 2 runs at one of two speeds on
    // a given output buffer: the same order on another allocation of the same size, or the same
    // buffer with every pair's tasks rotated by k/npairs of its range (order 2), takes the other
    // (64 x 20k: 18.5-20.2 vs 21.2-25.4 ms; which one is fast flips between the two orders;
    // profiles/r05_outbuf_probe.txt).  So the first two launches on an output buffer run orders 1
    // and 2 and time their pass 2 (HIP events; the second launch waits for the first's), and later
    // launches on that buffer take the faster.  GSA_EXPAND_RR fixes the order: 0 pair-major, 1, 2,
    // 3 shuffled, 4-6 probe variants.
    const int rrEnv = opt.rr >= 0 ? opt.rr : env_int(ctx, "GSA_EXPAND_RR", -1);
    int rr = rrEnv >= 0 ? rrEnv : 1;
    const bool tune = rrEnv < 0 && npairs > 1 && !fused;
    bool tuneRecord = false;
    if (tune)
    {
        if (xt.key != (const void*)pairs[0].score || xt.pairs != npairs || xt.tasks != tasks)
        {
            xt.key = (const void*)pairs[0].score;
            xt.pairs = npairs;
            xt.tasks = tasks;
            xt.ms[0] = xt.ms[1] = -1.f;
            xt.pending = false;
            xt.cold = true;
        }
        // (the tuning is best effort: an event that cannot be created or read ends it on order 1)
        bool evOk = true;
        for (int k = 0; k < 2; ++k)
            if (!xt.ev[k] && hipEventCreate(&xt.ev[k]) != hipSuccess)
            {
                xt.ev[k] = nullptr;
                evOk = false;
            }
        // the previous candidate's time, if its launch has ended: the host never waits for it (a
        // launch still running keeps the measurement pending and this one runs untimed)
        bool busy = false;
        if (xt.pending && evOk)
        {
            const hipError_t q = hipEventQuery(xt.ev[1]);
            float ms = -1.f;
            if (q == hipErrorNotReady)
            {
                (void)hipGetLastError();
                busy = true;
            }
            else if (q != hipSuccess || hipEventElapsedTime(&ms, xt.ev[0], xt.ev[1]) != hipSuccess || !(ms >= 0.f))
            {
                (void)hipGetLastError();
                evOk = false;
            }
            else
                xt.ms[xt.last] = ms;
            if (!busy) xt.pending = false;
        }
        if (!evOk)
        {
            xt.ms[0] = xt.ms[1] = 0.f;  // both "measured": order 1 from now on
            xt.pending = false;
        }
        const int next = xt.ms[0] < 0 ? 0 : xt.ms[1] < 0 ? 1 : (xt.ms[1] < xt.ms[0] ? 1 : 0);
        tuneRecord = !busy && !xt.cold && xt.ms[next] < 0;
        xt.cold = false;
        if (tuneRecord) xt.last = next;
        rr = next + 1;
    }
    // The schedule: runs of xRun tasks of one tile column of one pair, consecutive row chunks (a
    // workgroup claims a run; its tile waves rebuild the column profile only when the tile column
    // changes: the rebuild and its two barriers stop the workgroup's store stream, ~10 % of the
    // expansion at 100k one task at a time, profiles/r06_expand_probes.txt), padded with (-1, 0)
    // entries to whole runs.  Runs in order: a single pair by when their pass-1 rows arrive (the
    // fused fill; it helps two launches too), a batch round-robin over the pairs (rr 1; rr 2
    // rotated, 0 pair-major, 3 shuffled).
    // runs of 4 (8 and 16 measured equal at 100k, r06), shorter when the runs would not cover the
    // CUs twice: a 10k pair's 483 tasks were 121 runs of 4, one per workgroup, four tasks in a row
    // on half the CUs, and its last run alone set the fill's tail (48 us after the last strip)
    long long allTasks = 0;
    for (int p = 0; p < npairs; ++p) allTasks += (long long)ex[(size_t)p].rowChunks * ex[(size_t)p].colTiles;
    const long long cus = std::max(1, ctx->cu_count);
    const int xRun = allTasks >= 8 * cus ? 4 : allTasks >= 4 * cus ? 2 : 1;
    std::vector<int> xs;
    {
        struct Run { int p, g, jT; };
        auto runs_of = [&](int p) { return ((ex[(size_t)p].rowChunks + xRun - 1) / xRun) * ex[(size_t)p].colTiles; };
        auto run_at = [&](int p, long long r) { const int ct = ex[(size_t)p].colTiles; return Run {p, (int)(r / ct), (int)(r % ct)}; };
        std::vector<Run> order;
        if (npairs == 1)
        {
            // Task (rc, jT) can start once strip s1 = the last of its rows' strips has passed column
            // cb + cols + 64; strip s starts ~s lag steps after strip 0 and sweeps a column per
            // step, so it is ready at about s1 lag + cb + cols.  Row-chunk-major order made the first
            // workgroups wait for whole rows: at 100k they claimed row chunk 0's tiles to the far end
            // of the matrix, ready only ~4 ms later (profiles/r06_fused100k.txt).  lag = columns per
            // 256-row strip, GSA_FUSED_LAG (default 192: the 100k pair's strip-to-strip spacing).
            const gsa::ExpandPair& d = ex[0];
            constexpr long long lag = 192;
            const int cm = xWaves * xmt;
            std::vector<std::pair<long long, long long>> key;
            for (long long r = 0; r < runs_of(0); ++r)
            {
                const Run u = run_at(0, r);
                const long long s1 = std::min<long long>((cm * (u.g * xRun + 1) - 1) / 4, d.p1Strips - 1);
                key.push_back({s1 * lag + gsa::ex_cb(d, u.jT) + gsa::ex_cols(d, u.jT), r});
            }
            std::stable_sort(key.begin(), key.end());
            for (const auto& k : key) order.push_back(run_at(0, k.second));
        }
        else if (rr == 0)
        {
            for (int p = 0; p < npairs; ++p)
                for (long long r = 0; r < runs_of(p); ++r) order.push_back(run_at(p, r));
        }
        else
        {
            std::vector<int> ord((size_t)npairs);
            for (int p = 0; p < npairs; ++p) ord[(size_t)p] = p;
            std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return runs_of(x) > runs_of(y); });
            // rr 2: pair k of the order starts k / npairs of the way into its runs
            std::vector<long long> rot((size_t)npairs, 0);
            if (rr == 2)
                for (int k = 0; k < npairs; ++k)
                    rot[(size_t)ord[(size_t)k]] = runs_of(ord[(size_t)k]) * k / npairs;
            for (long long j = 0; j < runs_of(ord[0]); ++j)
                for (int k = 0; k < npairs; ++k)
                {
                    const int p = ord[(size_t)k];
                    if (runs_of(p) <= j) break;
                    order.push_back(run_at(p, (j + rot[(size_t)p]) % runs_of(p)));
                }
            if (rr == 3)
            {
                // the whole schedule shuffled (fixed seed)
                uint64_t z = 0x9e3779b97f4a7c15ull;
                for (size_t i = order.size(); i > 1; --i)
                {
                    z += 0x9e3779b97f4a7c15ull;
                    uint64_t q = z;
                    q = (q ^ (q >> 30)) * 0xbf58476d1ce4e5b9ull;
                    q = (q ^ (q >> 27)) * 0x94d049bb133111ebull;
                    q ^= q >> 31;
                    std::swap(order[i - 1], order[(size_t)(q % i)]);
                }
            }
        }
        xs.reserve(2 * order.size() * (size_t)xRun);
        for (const Run& u : order)
        {
            const gsa::ExpandPair& d = ex[(size_t)u.p];
            for (int i = 0; i < xRun; ++i)
            {
                const int rc = u.g * xRun + i;
                xs.push_back(rc < d.rowChunks ? u.p : -1);
                xs.push_back(rc < d.rowChunks ? rc * d.colTiles + u.jT : 0);
            }
        }
    }
    const long long nEntries = (long long)(xs.size() / 2);
    const size_t descBytes = ((size_t)npairs * sizeof(gsa::ExpandPair) + 15) & ~(size_t)15;
    const size_t exBytes = descBytes + xs.size() * sizeof(int);
    if (exdesc_cap < exBytes || !exdesc)
    {
        if (exdesc) (void)hipFree(exdesc);
        exdesc = nullptr;
        exdesc_cap = 0;
        if ((e = hipMalloc(&exdesc, std::max<size_t>(exBytes, 4096))) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        exdesc_cap = std::max<size_t>(exBytes, 4096);
    }
    const int slot = ctx->expin_next;
    ctx->expin_next = (slot + 1) % gsa_ctx::kStage;
    if (ctx->expin_used[slot] && (e = hipEventSynchronize(ctx->expin_ev[slot])) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (ctx->expin_cap[slot] < exBytes)
    {
        if (ctx->expin[slot]) (void)hipHostFree(ctx->expin[slot]);
        ctx->expin[slot] = nullptr;
        ctx->expin_cap[slot] = 0;
        if ((e = hipHostMalloc(&ctx->expin[slot], exBytes)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        ctx->expin_cap[slot] = exBytes;
    }
    std::memcpy(ctx->expin[slot], ex.data(), (size_t)npairs * sizeof(gsa::ExpandPair));
    if (!xs.empty()) std::memcpy((char*)ctx->expin[slot] + descBytes, xs.data(), xs.size() * sizeof(int));
    e = hipMemcpyAsync(exdesc, ctx->expin[slot], exBytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(ctx->expin_ev[slot], st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    ctx->expin_used[slot] = true;
    gsa::ExpandArgs xa {};
    xa.subst = subst;
    xa.substsz = substsz;
    xa.g = gapo;
    xa.pairs = (const gsa::ExpandPair*)exdesc;
    xa.nPairs = npairs;
    xa.nTasks = (int)nEntries;
    xa.run = xRun;
    xa.sched = (const int*)((char*)exdesc + descBytes);
    xa.spin = ctx->spin_ticks;
    xa.err = ctx->ctl + 1;
    // (a group of a split batch has a claim counter of its own: the two groups' expansions overlap)
    xa.counter = ctx->ctl + 8 + opt.slot;
    // the fused single pair: every workgroup takes pass-1 tickets first.  A large pair's expansion
    // fills HBM, and its strips hand row 64m to a storer wave (their own write-through stores stalled
    // them); a small one's keeps HBM idle enough for the strips to store it directly, without the
    // staging's ~5 % per step (nw_krow.hip nw_full_fused_kernel): 10k direct, 100k staged
    const int stagedKnob = env_int(ctx, "GSA_FUSED_STAGED", -1);  // (tests: both instances at every size)
    const bool staged = stagedKnob >= 0 ? stagedKnob != 0
                                        : (long long)(pairs[0].adjrows - 1) * (long long)(pairs[0].adjcols - 1) > (1ll << 30);
    const FusedLaunch fl {&xa, ns, gsa::kExpStreamWaves, 1 << 30, staged};
    const int xGrid = (int)std::max<long long>(1, std::min<long long>(ctx->cu_count, (nEntries + xRun - 1) / xRun));
    // gsa_set_full_timing: events before pass 1, between the passes and after pass 2, and the
    // expansion's clock stamps (one per workgroup)
    const bool timed = ctx->timing && !opt.split;
    if (!opt.split) ctx->timing_state = 0;
    if (timed && !fused)
    {
        if (ctx->clk_cap < (size_t)xGrid || !ctx->clk)
        {
            if (ctx->clk) (void)hipFree(ctx->clk);
            ctx->clk = nullptr;
            ctx->clk_cap = 0;
            if ((e = hipMalloc(&ctx->clk, (size_t)std::max(xGrid, 1024) * 8)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
            ctx->clk_cap = (size_t)std::max(xGrid, 1024);
        }
        xa.clk = ctx->clk;
        ctx->clk_n = (size_t)xGrid;
    }
    if (timed && (e = hipEventRecord(ctx->pev[0], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (opt.startEv && (e = hipEventRecord(opt.startEv, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (opt.beforeP1 && (e = hipStreamWaitEvent(st, opt.beforeP1, 0)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    int s = enqueue_batch(ctx, gsa::kModeSparse, npairs, p1.data(), subst, substsz, gapo, gsa::kExpHB, st, nullptr, 0,
                          nullptr, rows.data(), fused ? &fl : nullptr);
    if (s != GSA_SUCCESS) return s;
    if (fused)
    {
        if (timed && (e = hipEventRecord(ctx->pev[2], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
        ctx->timing_state = timed ? 2 : 0;
        return s;
    }
    if (timed && (e = hipEventRecord(ctx->pev[1], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (opt.afterP1 && (e = hipEventRecord(opt.afterP1, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (opt.timeP1 && (e = hipEventRecord(opt.timeP1, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if ((e = hipMemsetAsync(xa.counter, 0, 4, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    if (tuneRecord && (e = hipEventRecord(xt.ev[0], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if ((e = gsa::launch_expand_stream(xa, st, xGrid)) != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    note_launch(ctx);
    if (tuneRecord)
    {
        if ((e = hipEventRecord(xt.ev[1], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
        xt.pending = true;
    }
    if (timed)
    {
        if ((e = hipEventRecord(ctx->pev[2], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
        ctx->timing_state = 1;
    }
    return GSA_SUCCESS;
}

// full fills: the two-pass fill (same box: 10k 100 -> 141 GCUPS, 64 x 20k batch 1084 -> 1093-1102
// GCUPS, profiles/r04_twopass.txt); GSA_FULL_KERNEL=lane: the one-pass lane fill (nw_lane.hip)
bool full_twopass(const gsa_ctx* ctx)
{
    const char* e = knob(ctx, "GSA_FULL_KERNEL");
    return !(e && std::strcmp(e, "lane") == 0);
}

// A batch whose pass-1 tickets are k full rounds and a short last one, split in two groups: group A
// (k rounds of tickets) on the caller's stream, group B (the rest) on a high-priority stream behind
// A's pass 1.  B's pass 1 then runs on the CUs A's pass 1 leaves, while A's expansion takes the
// others, instead of the last round's idle CUs waiting for every pair's pass 1.  Whether that pays
// depends on the box: 64 x 20k pairs, 0.434 -> 0.49-0.52 of HBM peak on four boxes, 0.508 -> 0.475
// on another (profiles/r05_split_ab.txt), so enqueue_full times both on the batch's first launches.
struct SplitPlan
{
    std::vector<gsa_pair_dev> pa, pb;
    std::vector<int32_t> la, lb;
};
bool split_plan(gsa_ctx* ctx, int npairs, const gsa_pair_dev* pairs, const int32_t* lds, SplitPlan& sp)
{
    if (npairs < 2 || env_int(ctx, "GSA_FULL_FUSED", 1) >= 2) return false;
    long long tileRows = 0;
    for (int p = 0; p < npairs; ++p)
    {
        if (pairs[p].adjrows < 2 || pairs[p].adjcols < 2) return false;
        tileRows += std::max<long long>(1, ((long long)pairs[p].adjrows - 1 + gsa::kSparseTileBy - 1) / gsa::kSparseTileBy);
    }
    if (tileRows <= (long long)std::max(1, ctx->cu_count)) return false;  // 4-strip single round
    const int ns = env_int(ctx, "GSA_KROW_NS", 8) == 8 ? 8 : 4;
    std::vector<long long> t((size_t)npairs);
    long long T = 0;
    for (int p = 0; p < npairs; ++p)
    {
        gsa_sparse_geom geom;
        if (gsa_sparse_geometry(pairs[p].adjrows, pairs[p].adjcols, gsa::kExpHB, &geom) != GSA_SUCCESS) return false;
        t[(size_t)p] = gsa::krow_tickets(geom.tileHdrMatRows, ns, 4);
        T += t[(size_t)p];
    }
    const long long S = std::max(1, ctx->cu_count);  // (8, 4) XR workgroups: one per CU
    const long long k = T / S, tail = T - k * S;
    if (k < 1 || tail < 16 || tail > S - 16) return false;
    // group A: pairs by tickets, largest first, while they fit k rounds; B: the rest
    std::vector<int> ord((size_t)npairs);
    for (int p = 0; p < npairs; ++p) ord[(size_t)p] = p;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return t[(size_t)x] > t[(size_t)y]; });
    long long ta = 0;
    for (int p : ord)
    {
        const bool toA = ta + t[(size_t)p] <= k * S;
        if (toA) ta += t[(size_t)p];
        (toA ? sp.pa : sp.pb).push_back(pairs[p]);
        if (lds) (toA ? sp.la : sp.lb).push_back(lds[p]);
    }
    return !sp.pa.empty() && !sp.pb.empty();
}

// The two groups of a split plan; rr: both groups' expansion order (-1: each tuned on its own
// scratch slot); startEv: recorded on st before group A's pass 1.  Returns kNoScratch when nothing
// was enqueued (no room for group A's scratch).
int enqueue_full_split(gsa_ctx* ctx, const SplitPlan& sp, bool hasLds, const int32_t* subst, int32_t substsz,
                       int32_t gapo, hipStream_t st, int rr, hipEvent_t startEv)
{
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (!ctx->splitstream)
    {
        int lo = 0, hi = 0;
        if ((e = hipDeviceGetStreamPriorityRange(&lo, &hi)) != hipSuccess ||
            (e = hipStreamCreateWithPriority(&ctx->splitstream, hipStreamNonBlocking, hi)) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    }
    for (int q = 0; q < 2; ++q)
        if (!ctx->split_ev[q] && (e = hipEventCreateWithFlags(&ctx->split_ev[q], hipEventDisableTiming)) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    const bool timed = ctx->timing;
    if (timed && (e = hipEventRecord(ctx->pev[0], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    // B's stream waits for everything before this call on the caller's stream too
    if ((e = hipEventRecord(ctx->split_ev[1], st)) != hipSuccess ||
        (e = hipStreamWaitEvent(ctx->splitstream, ctx->split_ev[1], 0)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    TwoPassOpts oa, ob;
    oa.slot = 0;
    oa.afterP1 = ctx->split_ev[0];
    oa.timeP1 = timed ? ctx->pev[1] : nullptr;  // pass1_ms: group A's pass 1
    oa.startEv = startEv;
    oa.split = true;
    oa.rr = rr;
    ob.slot = 1;
    ob.beforeP1 = ctx->split_ev[0];
    ob.split = true;
    ob.rr = rr;
    int r = enqueue_full_twopass(ctx, (int)sp.pa.size(), sp.pa.data(), hasLds ? sp.la.data() : nullptr, subst, substsz,
                                 gapo, st, oa);
    if (r != GSA_SUCCESS) return r;  // (kNoScratch: nothing enqueued yet; the caller's fallback)
    r = enqueue_full_twopass(ctx, (int)sp.pb.size(), sp.pb.data(), hasLds ? sp.lb.data() : nullptr, subst, substsz,
                             gapo, ctx->splitstream, ob);
    if (r == kNoScratch)  // no room for a second scratch: group B on the one-pass lane fill
    {
        if ((e = hipStreamWaitEvent(ctx->splitstream, ctx->split_ev[0], 0)) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
        r = enqueue_batch(ctx, gsa::kModeFull, (int)sp.pb.size(), sp.pb.data(), subst, substsz, gapo, 0,
                          ctx->splitstream, nullptr, 0, hasLds ? sp.lb.data() : nullptr);
    }
    if (r != GSA_SUCCESS) return r;
    // the caller's stream waits for group B
    if ((e = hipEventRecord(ctx->split_ev[1], ctx->splitstream)) != hipSuccess ||
        (e = hipStreamWaitEvent(st, ctx->split_ev[1], 0)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    if (timed)
    {
        if ((e = hipEventRecord(ctx->pev[2], st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
        ctx->timing_state = 3;
        ctx->timing_groups = 2;
        ctx->clk_n = 0;
    }
    return GSA_SUCCESS;
}

uint64_t batch_key(int npairs, const gsa_pair_dev* pairs, const int32_t* lds)
{
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)npairs;
    auto mix = [&](uint64_t v) {
        h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        h *= 0xbf58476d1ce4e5b9ull;
        h ^= h >> 31;
    };
    for (int p = 0; p < npairs; ++p)
    {
        mix((uint64_t)(uintptr_t)pairs[p].score);
        mix(((uint64_t)(uint32_t)pairs[p].adjrows << 32) | (uint32_t)pairs[p].adjcols);
        mix(lds ? (uint64_t)(uint32_t)lds[p] : 0);
    }
    return h;
}

// Every full fill: the two-pass fill, or the lane fill (GSA_FULL_KERNEL=lane, or no room for the
// two-pass scratch); lds: row pitches (null: unpadded).
// A batch that splits (split_plan) runs, unless GSA_FULL_SPLIT or GSA_EXPAND_RR fix it, four
// candidates on its first four launches: one group with expansion order 1 and 2, two groups with
// order 1 and 2, each timed from just before pass 1 to the end on the caller's stream (HIP events;
// a launch waits on the host for the previous one's end event), and later launches of the same
// batch (pairs, shapes, output pointers) take the fastest.  Best effort like the order tuning: an
// event that cannot be created or read ends it on candidate 0.
int enqueue_full(gsa_ctx* ctx, int npairs, const gsa_pair_dev* pairs, const int32_t* lds, const int32_t* subst,
                 int32_t substsz, int32_t gapo, hipStream_t st)
{
    if (full_twopass(ctx))
    {
        const int spEnv = env_int(ctx, "GSA_FULL_SPLIT", -1), rrEnv = env_int(ctx, "GSA_EXPAND_RR", -1);
        SplitPlan sp;
        const bool can = spEnv != 0 && !(spEnv < 0 && rrEnv >= 0) && split_plan(ctx, npairs, pairs, lds, sp);
        if (can && spEnv > 0)
        {
            const int r = enqueue_full_split(ctx, sp, lds != nullptr, subst, substsz, gapo, st, -1, nullptr);
            if (r != kNoScratch) return r;
        }
        else if (can)
        {
            gsa_ctx::FTune& ft = ctx->ft;
            const uint64_t key = batch_key(npairs, pairs, lds);
            if (ft.key != key)
            {
                ft.key = key;
                ft.last = -1;
                for (float& m : ft.ms) m = -1.f;
                ft.pending = false;
                ft.cold = true;
            }
            bool evOk = true;
            for (int k = 0; k < 2; ++k)
                if (!ft.ev[k] && hipEventCreate(&ft.ev[k]) != hipSuccess)
                {
                    (void)hipGetLastError();
                    ft.ev[k] = nullptr;
                    evOk = false;
                }
            // the previous candidate's time if its launch has ended (never a host wait: a launch
            // still running keeps it pending, and this one runs untimed)
            bool busy = false;
            if (ft.pending && evOk)
            {
                const hipError_t q = hipEventQuery(ft.ev[1]);
                float ms = -1.f;
                if (q == hipErrorNotReady)
                {
                    (void)hipGetLastError();
                    busy = true;
                }
                else if (q != hipSuccess || hipEventElapsedTime(&ms, ft.ev[0], ft.ev[1]) != hipSuccess || !(ms >= 0.f))
                {
                    (void)hipGetLastError();
                    evOk = false;
                }
                else
                    ft.ms[ft.last] = ms;
                if (!busy) ft.pending = false;
            }
            if (!evOk)
            {
                for (float& m : ft.ms) m = 0.f;  // all "measured": candidate 0 from now on
                ft.pending = false;
            }
            int next = 0;
            while (next < 4 && ft.ms[next] >= 0.f) ++next;
            if (busy || ft.cold)
                next = 0;  // (untimed: the first launch on fresh buffers, or a measurement pending)
            else if (next == 4)
            {
                next = 0;
                for (int k = 1; k < 4; ++k)
                    if (ft.ms[k] < ft.ms[next]) next = k;
                ft.last = -1;
            }
            const bool rec = !busy && !ft.cold && ft.ms[next] < 0.f;
            ft.cold = false;
            const int rr = (next & 1) + 1;
            int r;
            if (next >= 2)
                r = enqueue_full_split(ctx, sp, lds != nullptr, subst, substsz, gapo, st, rr, rec ? ft.ev[0] : nullptr);
            else
            {
                TwoPassOpts o;
                o.rr = rr;
                o.startEv = rec ? ft.ev[0] : nullptr;
                r = enqueue_full_twopass(ctx, npairs, pairs, lds, subst, substsz, gapo, st, o);
            }
            if (r == GSA_SUCCESS && rec)
            {
                hipError_t e = hipEventRecord(ft.ev[1], st);
                if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
                ft.last = next;
                ft.pending = true;
            }
            if (r != kNoScratch) return r;
        }
        const int s = enqueue_full_twopass(ctx, npairs, pairs, lds, subst, substsz, gapo, st);
        if (s != kNoScratch) return s;
    }
    return enqueue_batch(ctx, gsa::kModeFull, npairs, pairs, subst, substsz, gapo, 0, st, nullptr, 0, lds);
}

}  // namespace

extern "C" {

const char* gsa_version(void) { return "gpuseqalign_amd 0.3 (gfx950 wavefront: K-rows sparse, two-pass full)"; }

int32_t gsa_sparse_tile_by(void) { return gsa::kSparseTileBy; }

int gsa_debug_stamps(gsa_ctx* ctx, uint64_t* out, int64_t cap, int64_t* n)
{
    if (!ctx || !n) return GSA_ERROR_INVALID_VALUE;
    *n = (int64_t)ctx->stamps_n;
    if (ctx->stamps_n == 0 || !out) return GSA_SUCCESS;
    if (cap < (int64_t)ctx->stamps_n) return GSA_ERROR_INVALID_VALUE;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stamps_stream);  // the launch's stream only
    if (e == hipSuccess) e = hipMemcpy(out, ctx->stamps, ctx->stamps_n * sizeof(uint64_t), hipMemcpyDeviceToHost);
    return e == hipSuccess ? GSA_SUCCESS : fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
}

int gsa_set_full_timing(gsa_ctx* ctx, int32_t on)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    if (on && !ctx->pev[0])
    {
        hipError_t e = hipSetDevice(ctx->device);
        for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreate(&ctx->pev[k]);
        if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    }
    ctx->timing = on != 0;
    ctx->timing_state = 0;
    return GSA_SUCCESS;
}

int gsa_last_full_timing(gsa_ctx* ctx, gsa_full_timing* out)
{
    if (!ctx || !out) return GSA_ERROR_INVALID_VALUE;
    std::memset(out, 0, sizeof(*out));
    out->pass1_ms = out->pass2_ms = -1.f;
    out->clock_ghz_median = out->clock_ghz_mean = -1.f;
    if (ctx->timing_state == 0) return GSA_ERROR_INVALID_VALUE;  // no timed full fill since timing was set
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipEventSynchronize(ctx->pev[2]);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    out->fused = ctx->timing_state == 2;
    out->groups = ctx->timing_state == 3 ? ctx->timing_groups : 0;
    if (out->fused) return hipEventElapsedTime(&out->pass2_ms, ctx->pev[0], ctx->pev[2]) == hipSuccess
                               ? GSA_SUCCESS : GSA_ERROR_CUDA_GENERAL;
    if (hipEventElapsedTime(&out->pass1_ms, ctx->pev[0], ctx->pev[1]) != hipSuccess ||
        hipEventElapsedTime(&out->pass2_ms, ctx->pev[1], ctx->pev[2]) != hipSuccess)
        return GSA_ERROR_CUDA_GENERAL;
    if (ctx->clk_n == 0) return GSA_SUCCESS;
    std::vector<unsigned long long> v(ctx->clk_n);
    if ((e = hipMemcpy(v.data(), ctx->clk, v.size() * 8, hipMemcpyDeviceToHost)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    std::vector<float> ghz;
    ghz.reserve(v.size());
    double cyc = 0, ticks = 0;
    for (unsigned long long w : v)
    {
        const double c = (double)(uint32_t)w, t = (double)(uint32_t)(w >> 32);
        if (t < 100) continue;  // under 1 us: too short to resolve
        ghz.push_back((float)(c / t * 0.1));
        cyc += c;
        ticks += t;
    }
    out->workgroups = (int64_t)ghz.size();
    if (ghz.empty()) return GSA_SUCCESS;
    std::nth_element(ghz.begin(), ghz.begin() + ghz.size() / 2, ghz.end());
    out->clock_ghz_median = ghz[ghz.size() / 2];
    out->clock_ghz_mean = (float)(cyc / ticks * 0.1);
    return GSA_SUCCESS;
}

int gsa_ctx_create(int device, gsa_ctx** out)
{
    if (!out) return GSA_ERROR_INVALID_VALUE;
    *out = nullptr;
    gsa_ctx* ctx = new (std::nothrow) gsa_ctx();
    if (!ctx) return GSA_ERROR_MEMORY_ALLOCATION;
    ctx->device = device;
    for (const char* k : kKnobNames)
        if (const char* v = std::getenv(k)) ctx->knobs[k] = v;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ctx->cu_count, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess)
    {
        int lm = 0;
        if (hipDeviceGetAttribute(&lm, hipDeviceAttributeSharedMemPerBlockOptin, device) == hipSuccess && lm > 0)
            ctx->lds_max = lm;
        else if (hipDeviceGetAttribute(&lm, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lm > 0)
            ctx->lds_max = lm;
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    // mlsppt's copy-back stream, created next so that it gets a hardware queue of its own
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->ptstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&ctx->ctl, 256);
    if (e == hipSuccess) e = hipMemset(ctx->ctl, 0, 256);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
    for (int k = 0; k < gsa_ctx::kStage && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&ctx->stage_ev[k], hipEventDisableTiming);
    for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&ctx->ptev[k], hipEventDisableTiming);
    for (int k = 0; k < gsa_ctx::kStage && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&ctx->expin_ev[k], hipEventDisableTiming);
    if (e != hipSuccess)
    {
        int code = (int)e;
        gsa_ctx_destroy(ctx);
        (void)code;
        return GSA_ERROR_CUDA_GENERAL;
    }
    *out = ctx;
    return GSA_SUCCESS;
}

void gsa_ctx_destroy(gsa_ctx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int k = 0; k < 5; k++)
        if (ctx->dbuf[k]) (void)hipFree(ctx->dbuf[k]);
    if (ctx->gran) (void)hipFree(ctx->gran);
    if (ctx->desc) (void)hipFree(ctx->desc);
    if (ctx->chk) (void)hipFree(ctx->chk);
    if (ctx->exbuf) (void)hipFree(ctx->exbuf);
    if (ctx->exdesc) (void)hipFree(ctx->exdesc);
    if (ctx->xdone) (void)hipFree(ctx->xdone);
    if (ctx->stamps) (void)hipFree(ctx->stamps);
    if (ctx->clk) (void)hipFree(ctx->clk);
    if (ctx->bidi) (void)hipFree(ctx->bidi);
    for (hipEvent_t ev : ctx->pev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& t : ctx->xt)
        for (hipEvent_t ev : t.ev)
            if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : ctx->split_ev)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : ctx->ft.ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->splitstream)
    {
        (void)hipStreamSynchronize(ctx->splitstream);
        (void)hipStreamDestroy(ctx->splitstream);
    }
    if (ctx->exbuf2) (void)hipFree(ctx->exbuf2);
    if (ctx->exdesc2) (void)hipFree(ctx->exdesc2);
    for (int k = 0; k < gsa_ctx::kStage; ++k)
    {
        if (ctx->expin[k]) (void)hipHostFree(ctx->expin[k]);
        if (ctx->expin_ev[k]) (void)hipEventDestroy(ctx->expin_ev[k]);
    }
    if (ctx->tmoves) (void)hipFree(ctx->tmoves);
    if (ctx->tres) (void)hipFree(ctx->tres);
    if (ctx->tdirs) (void)hipFree(ctx->tdirs);
    if (ctx->tband) (void)hipFree(ctx->tband);
    if (ctx->tlist) (void)hipFree(ctx->tlist);
    if (ctx->sbnd) (void)hipFree(ctx->sbnd);
    if (ctx->sctl) (void)hipFree(ctx->sctl);
    if (ctx->ptflags) (void)hipHostFree(ctx->ptflags);
    if (ctx->ptpin) (void)hipHostFree(ctx->ptpin);
    for (hipEvent_t ev : ctx->ptev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->ptstream) (void)hipStreamDestroy(ctx->ptstream);
    for (int k = 0; k < gsa_ctx::kStage; ++k)
    {
        if (ctx->stage[k]) (void)hipHostFree(ctx->stage[k]);
        if (ctx->stage_ev[k]) (void)hipEventDestroy(ctx->stage_ev[k]);
    }
    for (int k = 0; k < gsa_ctx::kCopyThreads; ++k)
    {
        if (ctx->xstream[k]) (void)hipStreamDestroy(ctx->xstream[k]);
        for (int j = 0; j < 2; ++j)
        {
            if (ctx->xstage[k][j]) (void)hipHostFree(ctx->xstage[k][j]);
            if (ctx->xev[k][j]) (void)hipEventDestroy(ctx->xev[k][j]);
        }
    }
    if (ctx->ctl) (void)hipFree(ctx->ctl);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int gsa_last_hip_error(const gsa_ctx* ctx) { return ctx ? ctx->last_hip_error : 0; }


int gsa_device_cu_count(const gsa_ctx* ctx) { return ctx ? ctx->cu_count : 0; }

int gsa_sparse_geometry(int32_t adjrows, int32_t adjcols, int32_t tileBx, gsa_sparse_geom* geom)
{
    if (!geom || adjrows < 1 || adjcols < 1) return GSA_ERROR_INVALID_VALUE;
    if (tileBx < 64 || tileBx % 16 != 0) return GSA_ERROR_INVALID_VALUE;
    const int64_t tBy = gsa::kSparseTileBy;
    // padded dims as nwalign_gpu9_mlsp_diagdiagdiag.cu:416-431 (empty sequences -> one tile)
    int64_t trows = ((int64_t)adjrows - 1 + tBy - 1) / tBy;
    int64_t tcols = ((int64_t)adjcols - 1 + tileBx - 1) / tileBx;
    trows = std::max<int64_t>(trows, 1);
    tcols = std::max<int64_t>(tcols, 1);
    geom->tileBx = tileBx;
    geom->tileBy = (int32_t)tBy;
    geom->tileHdrMatRows = (int32_t)trows;
    geom->tileHdrMatCols = (int32_t)tcols;
    geom->tileHrowLen = tileBx + 1;
    geom->tileHcolLen = (int32_t)tBy + 1;
    geom->hrowElems = trows * tcols * (tileBx + 1);
    geom->hcolElems = trows * tcols * (tBy + 1);
    return GSA_SUCCESS;
}

int gsa_fill_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                      const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score, void* stream)
{
    if (!ctx || !score) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_pair_dev p {seqY, adjrows, seqX, adjcols, score, nullptr, nullptr};
    return enqueue_full(ctx, 1, &p, nullptr, subst, substsz, gapo, pick_stream(ctx, stream));
}

int32_t gsa_full_pitch(int32_t adjcols)
{
    if (adjcols < 1) return 0;
    const int64_t ld = 32 * (((int64_t)adjcols - 1 + 31) / 32) + 1;
    return ld > INT32_MAX ? 0 : (int32_t)ld;  // no pitch fits int32 past 2^31 - 32 columns
}

int32_t gsa_full_base_offset(void) { return 31; }

int gsa_fill_full_pitched_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                              const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score, int32_t ld,
                              void* stream)
{
    if (!ctx || !score) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    if (ld < adjcols) return GSA_ERROR_INVALID_VALUE;
    gsa_pair_dev p {seqY, adjrows, seqX, adjcols, score, nullptr, nullptr};
    return enqueue_full(ctx, 1, &p, &ld, subst, substsz, gapo, pick_stream(ctx, stream));
}

int gsa_fill_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                        const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* hrow,
                        int32_t* hcol, void* stream)
{
    if (!ctx || !hrow || !hcol) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    return enqueue_fill(ctx, gsa::kModeSparse, seqY, adjrows, seqX, adjcols, subst, substsz, gapo, nullptr, tileBx,
                        hrow, hcol, pick_stream(ctx, stream));
}

int gsa_fill_full_batch_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* subst,
                            int32_t substsz, int32_t gapo, void* stream)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    return enqueue_full(ctx, npairs, pairs, nullptr, subst, substsz, gapo, pick_stream(ctx, stream));
}

int gsa_fill_full_batch_pitched_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* lds,
                                    const int32_t* subst, int32_t substsz, int32_t gapo, void* stream)
{
    if (!ctx || !lds) return GSA_ERROR_INVALID_VALUE;
    return enqueue_full(ctx, npairs, pairs, lds, subst, substsz, gapo, pick_stream(ctx, stream));
}

int gsa_fill_sparse_batch_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* subst,
                              int32_t substsz, int32_t gapo, int32_t tileBx, void* stream)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    return enqueue_batch(ctx, gsa::kModeSparse, npairs, pairs, subst, substsz, gapo, tileBx,
                         pick_stream(ctx, stream));
}

int gsa_sync(gsa_ctx* ctx, void* stream)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    const hipStream_t st = pick_stream(ctx, stream);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    unsigned err = 0;
    if ((e = take_err(ctx, st, &err)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    // a hand-off spin of ANY launch since the last sync gave up (the word is sticky)
    if (err != 0) return GSA_ERROR_KERNEL_FAILURE;
    return GSA_SUCCESS;
}

int gsa_mem_stats_get(const gsa_ctx* ctx, gsa_mem_stats* out)
{
    if (!ctx || !out) return GSA_ERROR_INVALID_VALUE;
    *out = ctx->mem;
    return GSA_SUCCESS;
}

int gsa_mem_stats_reset(gsa_ctx* ctx)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    ctx->mem = gsa_mem_stats {};
    return GSA_SUCCESS;
}

int gsa_set_lap_callback(gsa_ctx* ctx, gsa_lap_fn fn, void* user)
{
    if (!ctx) return GSA_ERROR_INVALID_VALUE;
    ctx->lap_fn = fn;
    ctx->lap_user = fn ? user : nullptr;
    return GSA_SUCCESS;
}

int gsa_set_knob(gsa_ctx* ctx, const char* name, const char* value)
{
    if (!ctx || !name || !knob_known(name)) return GSA_ERROR_INVALID_VALUE;
    if (value)
        ctx->knobs[name] = value;
    else
        ctx->knobs.erase(name);
    return GSA_SUCCESS;
}

int gsa_set_watchdog(gsa_ctx* ctx, int64_t microseconds)
{
    if (!ctx || microseconds < 0 || microseconds > 3600ll * 1000000ll) return GSA_ERROR_INVALID_VALUE;
    ctx->spin_ticks = (unsigned long long)microseconds * 100ull;  // s_memrealtime: 100 MHz
    return GSA_SUCCESS;
}

namespace {

// Device -> pageable host copy of a finished result (the caller's buffers of gsa_align_*).  A
// plain hipMemcpy into pageable memory runs at ~16 GB/s here (one staged stream); this splits
// the range over kCopyThreads threads, each streaming kCopyChunk pieces through two pinned
// buffers on its own stream, so the DMA and the host copies of different pieces overlap.
hipError_t copy_d2h(gsa_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    constexpr int T = gsa_ctx::kCopyThreads;
    constexpr size_t kC = gsa_ctx::kCopyChunk;
    hipError_t e = hipSuccess;
    // non-blocking streams: mlsppt copies finished tile rows while the fill still runs
    for (int k = 0; k < T && e == hipSuccess; ++k)
        if (!ctx->xstream[k]) e = hipStreamCreateWithFlags(&ctx->xstream[k], hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    if (bytes < 2 * kC)
    {
        e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->xstream[0]);
        return e == hipSuccess ? hipStreamSynchronize(ctx->xstream[0]) : e;
    }
    for (int k = 0; k < T && e == hipSuccess; ++k)
    {
        for (int j = 0; j < 2 && e == hipSuccess; ++j)
        {
            if (!ctx->xstage[k][j]) e = hipHostMalloc(&ctx->xstage[k][j], kC, hipHostMallocDefault);
            if (e == hipSuccess && !ctx->xev[k][j]) e = hipEventCreateWithFlags(&ctx->xev[k][j], hipEventDisableTiming);
        }
    }
    if (e != hipSuccess) return e;
    // thread k: bytes [lo, hi), chunk aligned
    const size_t nChunks = (bytes + kC - 1) / kC, perT = (nChunks + T - 1) / T;
    hipError_t errs[T];
    auto work = [&](int k) {
        hipError_t r = hipSetDevice(ctx->device);
        const size_t lo = std::min(bytes, (size_t)k * perT * kC), hi = std::min(bytes, (size_t)(k + 1) * perT * kC);
        const size_t n = (hi - lo + kC - 1) / kC;
        auto issue = [&](size_t i) {
            const size_t off = lo + i * kC, len = std::min(kC, hi - off);
            hipError_t q = hipMemcpyAsync(ctx->xstage[k][i & 1], (const char*)src + off, len, hipMemcpyDeviceToHost,
                                          ctx->xstream[k]);
            return q == hipSuccess ? hipEventRecord(ctx->xev[k][i & 1], ctx->xstream[k]) : q;
        };
        if (r == hipSuccess && n > 0) r = issue(0);
        for (size_t i = 0; r == hipSuccess && i < n; ++i)
        {
            // chunk i+1 goes into the other buffer, whose host copy (chunk i-1) is done
            if (i + 1 < n && (r = issue(i + 1)) != hipSuccess) break;
            if ((r = hipEventSynchronize(ctx->xev[k][i & 1])) != hipSuccess) break;
            const size_t off = lo + i * kC;
            std::memcpy((char*)dst + off, ctx->xstage[k][i & 1], std::min(kC, hi - off));
        }
        if (r != hipSuccess) (void)hipStreamSynchronize(ctx->xstream[k]);
        errs[k] = r;
    };
    std::vector<std::thread> th;
    th.reserve(T - 1);
    for (int k = 1; k < T; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& x : th) x.join();
    for (int k = 0; k < T; ++k)
        if (errs[k] != hipSuccess) return errs[k];
    return hipSuccess;
}

}  // namespace

int gsa_align_full(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                   const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score_out, int32_t* align_cost,
                   gsa_laps* laps)
{
    if (!ctx || !seqY || !seqX || !subst || !score_out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_laps L {};
    auto t = Clock::now();
    const size_t cells = (size_t)adjrows * (size_t)adjcols;
    if ((s = ensure_dev(ctx, 0, (size_t)adjrows * 4)) || (s = ensure_dev(ctx, 1, (size_t)adjcols * 4)) ||
        (s = ensure_dev(ctx, 2, (size_t)substsz * substsz * 4)) || (s = ensure_dev(ctx, 3, cells * 4)))
        return s;
    L.alloc = ms_since(t);
    lap(ctx, "align.alloc");
    hipError_t e;
    if ((e = hipMemcpyAsync(ctx->dbuf[0], seqY, (size_t)adjrows * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[1], seqX, (size_t)adjcols * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[2], subst, (size_t)substsz * substsz * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipStreamSynchronize(ctx->stream)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_dev = ms_since(t);
    lap(ctx, "align.cpy_dev");
    L.init_hdr = 0.f;  // headers are written by the fill launch itself
    lap(ctx, "align.init_hdr");
    (void)hipEventRecord(ctx->ev0, ctx->stream);
    s = gsa_fill_full_dev(ctx, (const int32_t*)ctx->dbuf[0], adjrows, (const int32_t*)ctx->dbuf[1], adjcols,
                          (const int32_t*)ctx->dbuf[2], substsz, gapo, (int32_t*)ctx->dbuf[3], ctx->stream);
    if (s != GSA_SUCCESS) return s;
    (void)hipEventRecord(ctx->ev1, ctx->stream);
    if ((s = gsa_sync(ctx, ctx->stream)) != GSA_SUCCESS) return s;
    L.calc = ms_since(t);
    lap(ctx, "align.calc");
    (void)hipEventElapsedTime(&L.calc_kernel_ms, ctx->ev0, ctx->ev1);
    if ((e = copy_d2h(ctx, score_out, ctx->dbuf[3], cells * 4)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_host = ms_since(t);
    lap(ctx, "align.cpy_host");
    if (align_cost) *align_cost = score_out[cells - 1];
    if (laps) *laps = L;
    return GSA_SUCCESS;
}

int gsa_align_sparse(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                     const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* hrow_out,
                     int32_t* hcol_out, gsa_sparse_geom* geom_out, int32_t* align_cost, gsa_laps* laps)
{
    if (!ctx || !seqY || !seqX || !subst || !hrow_out || !hcol_out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_sparse_geom geom;
    if ((s = gsa_sparse_geometry(adjrows, adjcols, tileBx, &geom)) != GSA_SUCCESS) return s;
    gsa_laps L {};
    auto t = Clock::now();
    if ((s = ensure_dev(ctx, 0, (size_t)adjrows * 4)) || (s = ensure_dev(ctx, 1, (size_t)adjcols * 4)) ||
        (s = ensure_dev(ctx, 2, (size_t)substsz * substsz * 4)) || (s = ensure_dev(ctx, 3, (size_t)geom.hrowElems * 4)) ||
        (s = ensure_dev(ctx, 4, (size_t)geom.hcolElems * 4)))
        return s;
    L.alloc = ms_since(t);
    lap(ctx, "align.alloc");
    hipError_t e;
    if ((e = hipMemcpyAsync(ctx->dbuf[0], seqY, (size_t)adjrows * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[1], seqX, (size_t)adjcols * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[2], subst, (size_t)substsz * substsz * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipStreamSynchronize(ctx->stream)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_dev = ms_since(t);
    lap(ctx, "align.cpy_dev");
    lap(ctx, "align.init_hdr");  // headers are written by the fill launch itself
    (void)hipEventRecord(ctx->ev0, ctx->stream);
    s = gsa_fill_sparse_dev(ctx, (const int32_t*)ctx->dbuf[0], adjrows, (const int32_t*)ctx->dbuf[1], adjcols,
                            (const int32_t*)ctx->dbuf[2], substsz, gapo, tileBx, (int32_t*)ctx->dbuf[3],
                            (int32_t*)ctx->dbuf[4], ctx->stream);
    if (s != GSA_SUCCESS) return s;
    (void)hipEventRecord(ctx->ev1, ctx->stream);
    if ((s = gsa_sync(ctx, ctx->stream)) != GSA_SUCCESS) return s;
    L.calc = ms_since(t);
    lap(ctx, "align.calc");
    (void)hipEventElapsedTime(&L.calc_kernel_ms, ctx->ev0, ctx->ev1);
    if ((e = copy_d2h(ctx, hrow_out, ctx->dbuf[3], (size_t)geom.hrowElems * 4)) ||
        (e = copy_d2h(ctx, hcol_out, ctx->dbuf[4], (size_t)geom.hcolElems * 4)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_host = ms_since(t);
    lap(ctx, "align.cpy_host");
    // align_cost from the last tile, as the reference does after its copy-back (:713-716);
    // the reference adds this to the align.calc lap.
    int32_t cost = gsa_sparse_align_cost(hrow_out, hcol_out, &geom, seqY, adjrows, seqX, adjcols, subst, substsz, gapo);
    L.calc += ms_since(t);
    lap(ctx, "align.calc");
    if (align_cost) *align_cost = cost;
    if (geom_out) *geom_out = geom;
    if (laps) *laps = L;
    return GSA_SUCCESS;
}

int gsa_check_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t gapo, const gsa_sparse_geom* geom,
                         const int32_t* hrow, const int32_t* hcol, gsa_check_result* out, void* stream)
{
    if (!ctx || !seqY || !seqX || !subst || !geom || !hrow || !hcol || !out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_sparse_geom g;
    if ((s = gsa_sparse_geometry(adjrows, adjcols, geom->tileBx, &g)) != GSA_SUCCESS) return s;
    if (std::memcmp(&g, geom, sizeof(g)) != 0) return GSA_ERROR_INVALID_VALUE;  // not this pair's geometry
    gsa::CheckArgs a {};
    a.seqY = seqY;
    a.seqX = seqX;
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    a.adjrows = adjrows;
    a.adjcols = adjcols;
    a.tBx = g.tileBx;
    a.tBy = g.tileBy;
    a.trows = g.tileHdrMatRows;
    a.tcols = g.tileHdrMatCols;
    a.hrowElems = g.hrowElems;
    a.hrow = hrow;
    a.hcol = hcol;
    return run_check(ctx, a, true, pick_stream(ctx, stream), out);
}

int gsa_check_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                       const int32_t* subst, int32_t substsz, int32_t gapo, const int32_t* score,
                       gsa_check_result* out, void* stream)
{
    if (!ctx || !seqY || !seqX || !subst || !score || !out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa::CheckArgs a {};
    a.seqY = seqY;
    a.seqX = seqX;
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    a.adjrows = adjrows;
    a.adjcols = adjcols;
    a.score = score;
    a.ld = adjcols;
    return run_check(ctx, a, false, pick_stream(ctx, stream), out);
}

int gsa_check_full_pitched_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX,
                               int32_t adjcols, const int32_t* subst, int32_t substsz, int32_t gapo,
                               const int32_t* score, int32_t ld, gsa_check_result* out, void* stream)
{
    if (!ctx || !seqY || !seqX || !subst || !score || !out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    if (ld < adjcols) return GSA_ERROR_INVALID_VALUE;
    gsa::CheckArgs a {};
    a.seqY = seqY;
    a.seqX = seqX;
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    a.adjrows = adjrows;
    a.adjcols = adjcols;
    a.score = score;
    a.ld = ld;
    return run_check(ctx, a, false, pick_stream(ctx, stream), out);
}

// NwHash1_Plain (nwtrace1_plain.cpp:133-154) over a matrix that stays in HBM.  djb2-xor is one serial
// chain over every cell in row-major order, so the host folds it while the DMA brings the next rows:
// row chunks (~64 MB, unpadded) alternate between two pinned buffers on the context's copy stream.
int gsa_hash_full_dev(gsa_ctx* ctx, const int32_t* score, int32_t adjrows, int32_t adjcols, int32_t ld,
                      uint32_t* hash, void* stream)
{
    if (!ctx || !score || !hash || adjrows < 1 || adjcols < 1 || ld < adjcols) return GSA_ERROR_INVALID_VALUE;
    hipError_t e = hipSetDevice(ctx->device);
    const hipStream_t st = pick_stream(ctx, stream);
    // (the caller's work on `stream` first: the matrix may still be being filled)
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    const int64_t rowsPer = std::max<int64_t>(1, ((int64_t)16 << 20) / adjcols);
    const int64_t nChunks = (adjrows + rowsPer - 1) / rowsPer;
    const size_t bufBytes = (size_t)std::min<int64_t>(rowsPer, adjrows) * (size_t)adjcols * 4;
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    int rc = GSA_SUCCESS;
    for (int k = 0; k < 2 && e == hipSuccess; ++k)
    {
        e = hipHostMalloc(&buf[k], bufBytes, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
    }
    auto issue = [&](int64_t c) {
        const int64_t r0 = c * rowsPer, n = std::min<int64_t>(rowsPer, adjrows - r0);
        hipError_t q = hipMemcpy2DAsync(buf[c & 1], (size_t)adjcols * 4, score + r0 * (int64_t)ld, (size_t)ld * 4,
                                        (size_t)adjcols * 4, (size_t)n, hipMemcpyDeviceToHost, st);
        return q == hipSuccess ? hipEventRecord(ev[c & 1], st) : q;
    };
    uint32_t h = 5381;
    if (e == hipSuccess) e = issue(0);
    for (int64_t c = 0; e == hipSuccess && c < nChunks; ++c)
    {
        if (c + 1 < nChunks && (e = issue(c + 1)) != hipSuccess) break;
        if ((e = hipEventSynchronize(ev[c & 1])) != hipSuccess) break;
        const uint32_t* v = (const uint32_t*)buf[c & 1];
        const int64_t n = std::min<int64_t>(rowsPer, adjrows - c * rowsPer) * adjcols;
        for (int64_t k = 0; k < n; ++k) h = ((h << 5) + h) ^ v[k];
    }
    if (e != hipSuccess)
    {
        (void)hipStreamSynchronize(st);
        rc = fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    }
    for (int k = 0; k < 2; ++k)
    {
        if (buf[k]) (void)hipHostFree(buf[k]);
        if (ev[k]) (void)hipEventDestroy(ev[k]);
    }
    if (rc == GSA_SUCCESS) *hash = h;
    return rc;
}

// NwTrace1_Plain (nwtrace1_plain.cpp:6-131) over a matrix that stays in HBM.  The walk reads three
// stored neighbours per move; it runs on the host over blocks of the matrix copied on demand
// (kTB rows x kTC columns ending at the walk's position, so a walk up and to the left stays inside
// a block for up to kTB / kTC moves), and its moves are folded as the device Trace2's are.
int gsa_trace_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                       const int32_t* score, int32_t ld, char* edit, int64_t cap, int64_t* edit_len,
                       uint32_t* trace_hash, int32_t* align_cost, void* stream)
{
    if (!ctx || !seqY || !seqX || !score || !edit || !edit_len || !trace_hash || adjrows < 1 || adjcols < 1 ||
        ld < adjcols)
        return GSA_ERROR_INVALID_VALUE;
    constexpr int64_t kTB = 1024, kTC = 2048;
    hipError_t e = hipSetDevice(ctx->device);
    const hipStream_t st = pick_stream(ctx, stream);
    std::vector<int32_t> Y((size_t)adjrows), X((size_t)adjcols);
    if (e == hipSuccess) e = hipMemcpyAsync(Y.data(), seqY, (size_t)adjrows * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(X.data(), seqX, (size_t)adjcols * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    int32_t* blk = nullptr;
    if ((e = hipHostMalloc((void**)&blk, (size_t)(kTB * kTC) * 4, hipHostMallocDefault)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    int64_t bi0 = -1, bj0 = 0, bh = 0, bw = 0;  // the block held: rows [bi0, bi0 + bh), columns [bj0, bj0 + bw)
    // make rows i-1..i and columns j-1..j resident (a block ending at (i, j))
    auto fetch = [&](int64_t i, int64_t j) {
        const int64_t i0 = std::max<int64_t>(0, i - kTB + 1), j0 = std::max<int64_t>(0, j - kTC + 1);
        const int64_t h = std::min<int64_t>(kTB, adjrows - i0), w = std::min<int64_t>(kTC, adjcols - j0);
        hipError_t q = hipMemcpy2DAsync(blk, (size_t)w * 4, score + i0 * (int64_t)ld + j0, (size_t)ld * 4,
                                        (size_t)w * 4, (size_t)h, hipMemcpyDeviceToHost, st);
        if (q == hipSuccess) q = hipStreamSynchronize(st);
        bi0 = i0;
        bj0 = j0;
        bh = h;
        bw = w;
        return q;
    };
    auto held = [&](int64_t i, int64_t j) {
        const int64_t ilo = i > 0 ? i - 1 : 0, jlo = j > 0 ? j - 1 : 0;
        return bi0 >= 0 && ilo >= bi0 && i < bi0 + bh && jlo >= bj0 && j < bj0 + bw;
    };
    auto at = [&](int64_t i, int64_t j) { return blk[(i - bi0) * bw + (j - bj0)]; };
    std::vector<unsigned char> moves;
    moves.reserve((size_t)(adjrows + adjcols));
    int64_t i = adjrows - 1, j = adjcols - 1;
    int32_t cost = 0;
    for (bool first = true; e == hipSuccess; first = false)
    {
        if (!held(i, j) && (e = fetch(i, j)) != hipSuccess) break;
        if (first) cost = at(i, j);
        // the reference's order: diagonal, then up if strictly greater, then left if strictly greater
        int64_t best = INT64_MIN;
        int di = 0, dj = 0;
        unsigned char m = 0;
        if (i > 0 && j > 0)
        {
            best = at(i - 1, j - 1);
            di = dj = -1;
            m = X[(size_t)j] == Y[(size_t)i] ? '=' : 'X';
        }
        if (i > 0 && best < at(i - 1, j))
        {
            best = at(i - 1, j);
            di = -1;
            dj = 0;
            m = 'I';
        }
        if (j > 0 && best < at(i, j - 1))
        {
            best = at(i, j - 1);
            di = 0;
            dj = -1;
            m = 'D';
        }
        if (di == 0 && dj == 0) break;
        moves.push_back(m);
        i += di;
        j += dj;
    }
    (void)hipHostFree(blk);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    if (align_cost) *align_cost = cost;
    return gsa::fold_moves(moves.data(), (int64_t)moves.size(), edit, cap, edit_len, trace_hash);
}

int gsa_trace_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t gapo, const gsa_sparse_geom* geom,
                         const int32_t* hrow, const int32_t* hcol, char* edit, int64_t cap, int64_t* edit_len,
                         uint32_t* trace_hash, int32_t* align_cost, void* stream)
{
    if (!ctx || !seqY || !seqX || !subst || !geom || !hrow || !hcol || !edit || !edit_len || !trace_hash)
        return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_sparse_geom g;
    if ((s = gsa_sparse_geometry(adjrows, adjcols, geom->tileBx, &g)) != GSA_SUCCESS) return s;
    if (std::memcmp(&g, geom, sizeof(g)) != 0) return GSA_ERROR_INVALID_VALUE;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    hipStream_t st = pick_stream(ctx, stream);
    // start: NwTrace2_GetTileAndElemIJ(adjrows-1, adjcols-1) with its saturation (nwtrace2_sparse.cpp:8-38)
    const int64_t i0 = adjrows - 1, j0 = adjcols - 1;
    int64_t iT = i0 / g.tileBy, jT = j0 / g.tileBx, iE = i0 % g.tileBy, jE = j0 % g.tileBx;
    if (iT == g.tileHdrMatRows) { iT -= 1; iE += g.tileBy; }
    if (jT == g.tileHdrMatCols) { jT -= 1; jE += g.tileBx; }
    const size_t nmax = (size_t)i0 + (size_t)j0 + 1;
    if (ctx->tmoves_cap < nmax)
    {
        if (ctx->tmoves) (void)hipFree(ctx->tmoves);
        ctx->tmoves = nullptr;
        ctx->tmoves_cap = 0;
        if ((e = hipMalloc(&ctx->tmoves, nmax)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        ctx->tmoves_cap = nmax;
    }
    if (!ctx->tres && (e = hipMalloc(&ctx->tres, 64)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    const bool dirs_lds = gsa::trace_lds_bytes(g.tileBy, g.tileBx, substsz, true) <= 160 * 1024;
    if (!dirs_lds)
    {
        const size_t bytes = gsa::trace_dir_words(g.tileBy, g.tileBx) * 4;
        if (ctx->tdirs_cap < bytes)
        {
            if (ctx->tdirs) (void)hipFree(ctx->tdirs);
            ctx->tdirs = nullptr;
            ctx->tdirs_cap = 0;
            if ((e = hipMalloc(&ctx->tdirs, bytes)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
            ctx->tdirs_cap = bytes;
        }
    }
    gsa::TraceArgs a {};
    a.seqY = seqY;
    a.seqX = seqX;
    a.subst = subst;
    a.substsz = substsz;
    a.g = gapo;
    a.adjrows = adjrows;
    a.adjcols = adjcols;
    a.tBx = g.tileBx;
    a.tBy = g.tileBy;
    a.tcols = g.tileHdrMatCols;
    a.hrow = hrow;
    a.hcol = hcol;
    a.iT0 = (int)iT;
    a.jT0 = (int)jT;
    a.iE0 = (int)iE;
    a.jE0 = (int)jE;
    a.edits = ctx->tmoves;
    a.cap = (long long)nmax;
    a.res = ctx->tres;
    a.dirs_scratch = dirs_lds ? nullptr : ctx->tdirs;
    // The walk enters tiles one after another, and recomputing one (a row scan over its rows) takes
    // ~160 us at 1024 x 256.  The tiles are independent given their headers, so the ones within
    // GSA_TRACE_BAND columns (default 1024) of the diagonal are recomputed first by many workgroups
    // at once; the walk copies their codes (or reads them in place when a tile is too wide for
    // LDS) and recomputes only the tiles it finds outside the band.
    a.tmap = nullptr;
    a.tcodes = nullptr;
    // The band is only a speed-up: its codes take at most 512 MB and half the free device memory
    // (GSA_TRACE_BAND_BUDGET, bytes, lowers the cap), and if its buffers cannot be had the walk
    // runs alone and recomputes every tile it enters.
    {
        const int band = env_int(ctx, "GSA_TRACE_BAND", 1024);
        const int trows = g.tileHdrMatRows, tcols = g.tileHdrMatCols;
        const size_t words = gsa::trace_dir_words(g.tileBy, g.tileBx);
        size_t budget = (size_t)512 << 20;
        {
            size_t freeB = 0, totalB = 0;
            if (hipMemGetInfo(&freeB, &totalB) == hipSuccess) budget = std::min(budget, freeB / 2);
            const char* eb = knob(ctx, "GSA_TRACE_BAND_BUDGET");
            if (eb) budget = std::min(budget, (size_t)std::strtoull(eb, nullptr, 10));
        }
        const size_t maxSlots = budget / (words * 4);
        std::vector<int> list, map((size_t)trows * (size_t)tcols, -1);
        const double slope = (double)std::max<int64_t>(1, adjcols - 1) / (double)std::max<int64_t>(1, adjrows - 1);
        for (int r = 0; band > 0 && r < trows && list.size() / 2 < maxSlots; ++r)
        {
            const double c0 = (double)r * g.tileBy * slope - band, c1 = (double)(r + 1) * g.tileBy * slope + band;
            const int j0 = std::max(0, (int)(c0 / g.tileBx)), j1 = std::min(tcols - 1, (int)(c1 / g.tileBx));
            for (int c = j0; c <= j1 && list.size() / 2 < maxSlots; ++c)
            {
                if (r == iT && c == jT) continue;  // the start tile: recomputed by the walk (align cost)
                map[(size_t)r * tcols + c] = (int)(list.size() / 2);
                list.push_back(r);
                list.push_back(c);
            }
        }
        const int n = (int)(list.size() / 2);
        bool have = n > 0;
        const size_t ints = list.size() + map.size(), cbytes = (size_t)n * words * 4;
        if (have && ctx->tlist_cap < ints)
        {
            if (ctx->tlist) (void)hipFree(ctx->tlist);
            ctx->tlist = nullptr;
            ctx->tlist_cap = 0;
            if (hipMalloc(&ctx->tlist, ints * 4) == hipSuccess)
                ctx->tlist_cap = ints;
            else
                have = false;
        }
        if (have && ctx->tband_cap < cbytes)
        {
            if (ctx->tband) (void)hipFree(ctx->tband);
            ctx->tband = nullptr;
            ctx->tband_cap = 0;
            if (hipMalloc(&ctx->tband, cbytes) == hipSuccess)
                ctx->tband_cap = cbytes;
            else
                have = false;
        }
        if (!have) (void)hipGetLastError();  // a failed band allocation: the walk runs alone
        if (have)
        {
            // pageable sources: the copies are complete when the calls return
            if ((e = hipMemcpyAsync(ctx->tlist, list.data(), list.size() * 4, hipMemcpyHostToDevice, st)) != hipSuccess ||
                (e = hipMemcpyAsync(ctx->tlist + list.size(), map.data(), map.size() * 4, hipMemcpyHostToDevice, st)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
            a.tmap = ctx->tlist + list.size();
            a.tcodes = ctx->tband;
            if ((e = gsa::launch_trace_band(a, ctx->tlist, n, 4 * ctx->cu_count, st)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
        }
    }
    if ((e = gsa::launch_trace_sparse(a, st)) != hipSuccess) return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    long long res[2] = {0, 0};
    if ((e = hipMemcpyAsync(res, ctx->tres, sizeof(res), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    if (res[0] < 0 || (size_t)res[0] > nmax) return GSA_ERROR_INVALID_RESULT;
    std::vector<unsigned char> moves((size_t)res[0]);
    if (res[0] > 0 && (e = hipMemcpy(moves.data(), ctx->tmoves, (size_t)res[0], hipMemcpyDeviceToHost)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    if (align_cost) *align_cost = (int32_t)res[1];
    return gsa::fold_moves(moves.data(), (int64_t)res[0], edit, cap, edit_len, trace_hash);
}

}  // extern "C"

namespace {

// Largest |substitution value| (>= 1) of a host table.
long long subst_absmax(const int32_t* sub, int32_t substsz)
{
    long long smax = 1;
    for (size_t k = 0; k < (size_t)substsz * (size_t)substsz; ++k)
        smax = std::max<long long>(smax, sub[k] < 0 ? -(long long)sub[k] : (long long)sub[k]);
    return smax;
}

// gsa_score_dev; smax < 0: read the table back from the device (in stream order, so the caller's
// writes to it are seen) to find the largest |value|; gsa_score passes it from its host copy.
int score_dev_impl(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                   const int32_t* subst, int32_t substsz, int32_t gapo, int32_t gape, int32_t local,
                   gsa_score_result* out, hipStream_t st, long long smax)
{
    if (!ctx || !seqY || !seqX || !subst || !out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    if (gapo > gape || gape > 0) return GSA_ERROR_INVALID_VALUE;  // go <= ge <= 0 (nw_scan.hip)
    const int64_t R = adjrows - 1, C = adjcols - 1;
    out->calc_kernel_ms = 0.f;
    if (R == 0 || C == 0)
    {
        // one boundary: nothing to fill (score_oracle.c semantics)
        const int64_t k = R + C;
        out->score = (local || k == 0) ? 0 : (int32_t)(gapo + (k - 1) * gape);
        out->i_end = local ? 0 : R;
        out->j_end = local ? 0 : C;
        return GSA_SUCCESS;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    // value ranges: the largest |substitution value| bounds every score and shifted value
    if (smax < 0)
    {
        std::vector<int32_t> sub((size_t)substsz * (size_t)substsz);
        if ((e = hipMemcpyAsync(sub.data(), subst, sub.size() * 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
        smax = subst_absmax(sub.data(), substsz);
    }
    const long long span = (R + C) * (long long)(-gape) + (long long)(gape - gapo) + smax;
    // unshifted int32 (row scan): |H| <= smax*min(R,C) + |go| + (R+C)|ge|
    if (smax * std::min(R, C) + (long long)(-gapo) + (R + C) * (long long)(-gape) >= (1ll << 30))
        return GSA_ERROR_INVALID_VALUE;
    const int bits = sw_idx_bits(R, C);
    const long long scoreBound = std::min<long long>((1ll << 31) - 1, smax * std::min(R, C));
    const int scoreBits = scoreBound > 0 ? 64 - __builtin_clzll((unsigned long long)scoreBound) : 1;
    // SW end-cell keys (score << bits | ~index) must fit 64 bits: the row scan packs full scores
    if (local && bits + scoreBits > 63) return GSA_ERROR_INVALID_VALUE;
    // the strip kernel's SW mode needs go < 0 (cells past C then never tie the maximum) and scores
    // below 2^26 packed with bits index bits (it reports larger ones); both modes keep shifted
    // values (i+j)*ge apart within int32 with margin; otherwise the row scan
    // (and scores below 2^26 by construction, so that no shifted key can wrap before the kernel flags it)
    const bool stripOk = (!local || (gapo < 0 && bits + 27 <= 63 && smax * std::min(R, C) < (1ll << 26))) && span < (1ll << 28);
    if (!score_scan_forced(ctx) && stripOk)
    {
        s = score_ag_strip(ctx, seqY, R, seqX, C, subst, substsz, gapo, gape, local, out, st);
        if (s != kScoreTooLarge) return s;
    }
    const int64_t nTR = (R + 63) / 64;
    const size_t bnd = (size_t)(nTR + 1) * (size_t)(C + 1);
    const size_t need = 2 * bnd + (size_t)(nTR + 1);  // bh, bf, prog
    if (ctx->sbnd_cap < need)
    {
        if (ctx->sbnd) (void)hipFree(ctx->sbnd);
        ctx->sbnd = nullptr;
        ctx->sbnd_cap = 0;
        if ((e = hipMalloc(&ctx->sbnd, need * sizeof(int))) != hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        ctx->sbnd_cap = need;
    }
    if (!ctx->sctl && (e = hipMalloc(&ctx->sctl, 64)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
    gsa::ScoreArgs a {};
    a.seqY = seqY;
    a.seqX = seqX;
    a.subst = subst;
    a.substsz = substsz;
    a.go = gapo;
    a.ge = gape;
    a.R = R;
    a.C = C;
    a.nTR = (int)nTR;
    a.bh = ctx->sbnd;
    a.bf = ctx->sbnd + bnd;
    a.prog = ctx->sbnd + 2 * bnd;
    a.ticket = (unsigned*)ctx->sctl;
    a.err = (unsigned*)ctx->sctl + 1;
    a.spin = ctx->spin_ticks;
    a.best = ctx->sctl + 1;
    a.idxBits = sw_idx_bits(R, C);
    a.result = (int*)(ctx->sctl + 2);
    if ((e = hipMemsetAsync(a.prog, 0, (size_t)(nTR + 1) * sizeof(int), st)) != hipSuccess ||
        (e = hipMemsetAsync(ctx->sctl, 0, 64, st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    (void)hipEventRecord(ctx->ev0, st);
    if ((e = gsa::launch_score_scan(a, local, ctx->cu_count, st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    (void)hipEventRecord(ctx->ev1, st);
    unsigned long long ctl[3];
    if ((e = hipMemcpyAsync(ctl, ctx->sctl, sizeof(ctl), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_KERNEL_FAILURE);
    (void)hipEventElapsedTime(&out->calc_kernel_ms, ctx->ev0, ctx->ev1);
    if ((unsigned)(ctl[0] >> 32) != 0) return GSA_ERROR_KERNEL_FAILURE;  // a wait gave up
    if (local)
    {
        const int bits = sw_idx_bits(R, C);
        const unsigned long long mask = (1ull << bits) - 1;
        const unsigned long long idx = mask - (ctl[1] & mask);
        out->score = (int32_t)(ctl[1] >> bits);
        out->i_end = (int64_t)(idx / (unsigned long long)(C + 1));
        out->j_end = (int64_t)(idx % (unsigned long long)(C + 1));
    }
    else
    {
        out->score = (int32_t)(uint32_t)ctl[2];
        out->i_end = R;
        out->j_end = C;
    }
    return GSA_SUCCESS;
}

}  // namespace

extern "C" {

int gsa_score_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                  const int32_t* subst, int32_t substsz, int32_t gapo, int32_t gape, int32_t local,
                  gsa_score_result* out, void* stream)
{
    return score_dev_impl(ctx, seqY, adjrows, seqX, adjcols, subst, substsz, gapo, gape, local, out,
                          pick_stream(ctx, stream), -1);
}

int gsa_score(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
              const int32_t* subst, int32_t substsz, int32_t gapo, int32_t gape, int32_t local,
              gsa_score_result* out, gsa_laps* laps)
{
    if (!ctx || !seqY || !seqX || !subst || !out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_laps L {};
    auto t = Clock::now();
    if ((s = ensure_dev(ctx, 0, (size_t)adjrows * 4)) || (s = ensure_dev(ctx, 1, (size_t)adjcols * 4)) ||
        (s = ensure_dev(ctx, 2, (size_t)substsz * substsz * 4)))
        return s;
    L.alloc = ms_since(t);
    lap(ctx, "align.alloc");
    hipError_t e;
    if ((e = hipMemcpyAsync(ctx->dbuf[0], seqY, (size_t)adjrows * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[1], seqX, (size_t)adjcols * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[2], subst, (size_t)substsz * substsz * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipStreamSynchronize(ctx->stream)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_dev = ms_since(t);
    lap(ctx, "align.cpy_dev");
    s = score_dev_impl(ctx, (const int32_t*)ctx->dbuf[0], adjrows, (const int32_t*)ctx->dbuf[1], adjcols,
                       (const int32_t*)ctx->dbuf[2], substsz, gapo, gape, local, out, ctx->stream,
                       subst_absmax(subst, substsz));
    if (s != GSA_SUCCESS) return s;
    L.calc = ms_since(t);
    lap(ctx, "align.calc");
    L.calc_kernel_ms = out->calc_kernel_ms;
    if (laps) *laps = L;
    return GSA_SUCCESS;
}

int gsa_align_sparse_pt(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                        const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* hrow_out,
                        int32_t* hcol_out, gsa_sparse_geom* geom_out, int32_t* align_cost, gsa_laps* laps)
{
    if (!ctx || !seqY || !seqX || !subst || !hrow_out || !hcol_out) return GSA_ERROR_INVALID_VALUE;
    int s = check_inputs(adjrows, adjcols, substsz);
    if (s != GSA_SUCCESS) return s;
    gsa_sparse_geom geom;
    if ((s = gsa_sparse_geometry(adjrows, adjcols, tileBx, &geom)) != GSA_SUCCESS) return s;
    gsa_laps L {};
    auto t = Clock::now();
    const size_t trows = (size_t)geom.tileHdrMatRows;
    if ((s = ensure_dev(ctx, 0, (size_t)adjrows * 4)) || (s = ensure_dev(ctx, 1, (size_t)adjcols * 4)) ||
        (s = ensure_dev(ctx, 2, (size_t)substsz * substsz * 4)) || (s = ensure_dev(ctx, 3, (size_t)geom.hrowElems * 4)) ||
        (s = ensure_dev(ctx, 4, (size_t)geom.hcolElems * 4)))
        return s;
    hipError_t e;
    if (ctx->ptflags_cap < trows)
    {
        if (ctx->ptflags) (void)hipHostFree(ctx->ptflags);
        ctx->ptflags = nullptr;
        ctx->ptflags_cap = 0;
        if ((e = hipHostMalloc((void**)&ctx->ptflags, trows * sizeof(unsigned long long), hipHostMallocMapped)) !=
            hipSuccess)
            return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
        std::memset(ctx->ptflags, 0, trows * sizeof(unsigned long long));
        ctx->ptflags_cap = trows;
    }
    unsigned long long* dflags = nullptr;
    if ((e = hipHostGetDevicePointer((void**)&dflags, ctx->ptflags, 0)) != hipSuccess)
        return fail(ctx, e, GSA_ERROR_CUDA_GENERAL);
    L.alloc = ms_since(t);
    lap(ctx, "align.alloc");
    if ((e = hipMemcpyAsync(ctx->dbuf[0], seqY, (size_t)adjrows * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[1], seqX, (size_t)adjcols * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->dbuf[2], subst, (size_t)substsz * substsz * 4, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipStreamSynchronize(ctx->stream)))
        return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_dev = ms_since(t);
    lap(ctx, "align.cpy_dev");
    lap(ctx, "align.init_hdr");  // headers are written by the fill launch itself
    int32_t* dhr = (int32_t*)ctx->dbuf[3];
    int32_t* dhc = (int32_t*)ctx->dbuf[4];
    // Column chunks of ptChunk tile columns: a chunk's headers (header rows and columns of every
    // tile row) are final once every tile row's word counts it; the fill reaches a column in every
    // super-strip within the wavefront's fill-in, so chunks complete left to right while the fill
    // runs, and each is copied back (one strided copy per matrix) as soon as it is complete.
    const int tcols = geom.tileHdrMatCols;
    // ~4096 columns per chunk, fewer (down to one tile column) while two chunks of every tile row
    // overfill the kPtPin staging slots: the pinned buffer stays 64 MB up to ~7.8M rows at tBx 64
    const size_t chunkCol = trows * (size_t)(geom.tileHrowLen + geom.tileHcolLen) * 4;  // one tile column
    int cw = std::max(1, std::min(tcols, (4096 + tileBx - 1) / tileBx));
    while (cw > 1 && 2 * chunkCol * (size_t)cw > gsa_ctx::kPtPin) cw = (cw + 1) / 2;
    const int nCh = (tcols + cw - 1) / cw;
    {
        // room for a batch of at least one chunk
        const size_t need = std::max(gsa_ctx::kPtPin, 2 * chunkCol * (size_t)cw);
        if (ctx->ptpin_cap < need)
        {
            if (ctx->ptpin) (void)hipHostFree(ctx->ptpin);
            ctx->ptpin = nullptr;
            ctx->ptpin_cap = 0;
            if ((e = hipHostMalloc(&ctx->ptpin, need, hipHostMallocDefault)) != hipSuccess)
                return fail(ctx, e, GSA_ERROR_MEMORY_ALLOCATION);
            ctx->ptpin_cap = need;
        }
    }
    (void)hipEventRecord(ctx->ev0, ctx->stream);
    s = enqueue_fill(ctx, gsa::kModeSparse, (const int32_t*)ctx->dbuf[0], adjrows, (const int32_t*)ctx->dbuf[1],
                     adjcols, (const int32_t*)ctx->dbuf[2], substsz, gapo, nullptr, tileBx, dhr, dhc, ctx->stream,
                     dflags, cw);
    if (s != GSA_SUCCESS) return s;
    (void)hipEventRecord(ctx->ev1, ctx->stream);
    const unsigned long long epoch = ctx->epoch;
    const size_t rowW = (size_t)geom.tileHrowLen * 4, rowH = (size_t)geom.tileHcolLen * 4;  // bytes per tile
    // The caller's result buffers are usually fresh pages: fault them in (the kernel zero-fills each
    // page on first touch) on the copy threads while the fill runs, before the first chunk arrives,
    // instead of inside the first chunk's scatter (measured: 2-4.6 ms for an 8 MB chunk at 100k)
    std::vector<std::thread> prefault;
    {
        constexpr int T = gsa_ctx::kCopyThreads;
        const size_t nb[2] = {(size_t)geom.hrowElems * 4, (size_t)geom.hcolElems * 4};
        char* base[2] = {(char*)hrow_out, (char*)hcol_out};
        for (int k = 0; k < T; ++k)
            prefault.emplace_back([=]() {
                for (int m = 0; m < 2; ++m)
                {
                    const size_t lo = nb[m] * k / T, hi = nb[m] * (k + 1) / T;
                    for (size_t o = lo & ~(size_t)4095; o < hi; o += 4096)
                        if (o >= lo) ((volatile char*)base[m])[o] = 0;
                }
            });
    }
    auto join_prefault = [&]() {
        for (auto& x : prefault) x.join();
        prefault.clear();
    };
    struct JoinAtExit  // every return path joins the prefault threads
    {
        std::vector<std::thread>& v;
        ~JoinAtExit()
        {
            for (auto& x : v)
                if (x.joinable()) x.join();
        }
    } joinAtExit {prefault};
    int copied = 0;  // chunks copied back
    // Two pinned slots: the strided DMA of one batch of chunks (ptstream) runs while the copy
    // threads scatter the previous batch into the tile-major host matrices.
    const size_t chunkBytes = trows * (size_t)cw * (rowW + rowH);
    const size_t slotBytes = ctx->ptpin_cap / 2;
    const int perBatch = (int)std::max<size_t>(1, slotBytes / chunkBytes);
    struct Batch
    {
        int c0, c1, slot;
    };
    Batch inflight[2];
    int nInflight = 0, issued = 0, nextSlot = 0;
    struct DrainAtExit  // an error return waits for DMAs still writing the pinned slots
    {
        gsa_ctx* c;
        const int& n;
        ~DrainAtExit()
        {
            if (n > 0) (void)hipStreamSynchronize(c->ptstream);
        }
    } drainAtExit {ctx, nInflight};
    auto batch_geom = [&](const Batch& bt, size_t& j0, size_t& wr, size_t& wc, char*& hh, char*& hc) {
        j0 = (size_t)bt.c0 * cw;
        const size_t j1 = std::min((size_t)tcols, (size_t)bt.c1 * cw);
        wr = (j1 - j0) * rowW;  // bytes per tile row
        wc = (j1 - j0) * rowH;
        hh = (char*)ctx->ptpin + (size_t)bt.slot * slotBytes;
        hc = hh + trows * wr;
    };
    // the DMA engine reads HBM (the fill's header stores are system-scope and acknowledged before
    // their chunk is published); ptstream is the context's second stream, created right after the
    // fill's, so it has a hardware queue of its own and its copies run beside the fill (copies on
    // streams that share the fill's queue wait for it: measured)
    auto issue = [&](int upTo) -> hipError_t {
        Batch bt {issued, std::min(upTo, issued + perBatch), nextSlot};
        size_t j0, wr, wc;
        char *hh, *hc;
        batch_geom(bt, j0, wr, wc, hh, hc);
        hipError_t err = hipMemcpy2DAsync(hh, wr, (const char*)dhr + j0 * rowW, tcols * rowW, wr, trows,
                                          hipMemcpyDeviceToHost, ctx->ptstream);
        if (err == hipSuccess)
            err = hipMemcpy2DAsync(hc, wc, (const char*)dhc + j0 * rowH, tcols * rowH, wc, trows, hipMemcpyDeviceToHost,
                                   ctx->ptstream);
        if (err == hipSuccess) err = hipEventRecord(ctx->ptev[bt.slot], ctx->ptstream);
        if (err != hipSuccess) return err;
        inflight[nInflight++] = bt;
        issued = bt.c1;
        nextSlot ^= 1;
        return hipSuccess;
    };
    // scatter the oldest batch once its DMA is done (wait: block until it is)
    auto scatter = [&](bool wait) -> hipError_t {
        const Batch bt = inflight[0];
        hipError_t err = wait ? hipEventSynchronize(ctx->ptev[bt.slot]) : hipEventQuery(ctx->ptev[bt.slot]);
        if (err == hipErrorNotReady) return hipSuccess;
        if (err != hipSuccess) return err;
        join_prefault();
        size_t j0, wr, wc;
        char *hh, *hc;
        batch_geom(bt, j0, wr, wc, hh, hc);
        constexpr int T = gsa_ctx::kCopyThreads;
        auto work = [&](int k) {
            for (size_t r = (size_t)k; r < trows; r += T)
            {
                std::memcpy((char*)hrow_out + r * tcols * rowW + j0 * rowW, hh + r * wr, wr);
                std::memcpy((char*)hcol_out + r * tcols * rowH + j0 * rowH, hc + r * wc, wc);
            }
        };
        std::vector<std::thread> th;
        for (int k = 1; k < T; ++k) th.emplace_back(work, k);
        work(0);
        for (auto& x : th) x.join();
        copied = bt.c1;
        inflight[0] = inflight[1];
        --nInflight;
        return hipSuccess;
    };
    // one pipeline step: issue a DMA for ready chunks if a slot is free, scatter a finished batch
    auto pump = [&](int ready, bool wait) -> hipError_t {
        hipError_t err = hipSuccess;
        if (ready > issued && nInflight < 2) err = issue(ready);
        if (err == hipSuccess && nInflight > 0) err = scatter(wait || nInflight == 2);
        return err;
    };
    for (;;)
    {
        const hipError_t q = hipStreamQuery(ctx->stream);  // the fill (and its headers kernel) finished?
        if (q != hipSuccess && q != hipErrorNotReady) return fail(ctx, q, GSA_ERROR_KERNEL_FAILURE);
        if (q == hipSuccess) break;
        int ready = nCh;
        for (size_t r = 0; r < trows && ready > issued; ++r)
        {
            const unsigned long long v = __atomic_load_n(ctx->ptflags + r, __ATOMIC_ACQUIRE);
            ready = std::min(ready, (v >> 32) == epoch ? (int)(v & 0xffffffffu) : 0);
        }
        if (ready > issued || nInflight > 0)
        {
            if ((e = pump(ready, false)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
        }
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if ((s = gsa_sync(ctx, ctx->stream)) != GSA_SUCCESS) return s;
    L.calc = ms_since(t);
    lap(ctx, "align.calc");
    (void)hipEventElapsedTime(&L.calc_kernel_ms, ctx->ev0, ctx->ev1);
    while (copied < nCh)
        if ((e = pump(nCh, true)) != hipSuccess) return fail(ctx, e, GSA_ERROR_MEMORY_TRANSFER);
    L.cpy_host = ms_since(t);
    lap(ctx, "align.cpy_host");
    int32_t cost = gsa_sparse_align_cost(hrow_out, hcol_out, &geom, seqY, adjrows, seqX, adjcols, subst, substsz, gapo);
    L.calc += ms_since(t);
    lap(ctx, "align.calc");
    if (align_cost) *align_cost = cost;
    if (geom_out) *geom_out = geom;
    if (laps) *laps = L;
    return GSA_SUCCESS;
}

}  // extern "C"
