// nwalign_amd.cpp -- the NwAlignFn adapters of the MI355X engine: the file a GpuSeqAlign
// maintainer adds to the reference, compiled here against this
// repository's mirror of the reference's types (nw_host.hpp) and linked into gsa_nw.
//
// Each adapter fills the outputs the reference's driver and consumers read from an align slot
// (NwAlignFn, src/nw_algorithm.hpp:11):
//   plain family  -> nw.score, res.align_cost                      (nwalign_gpu3_ml_diagdiag.cu:288-596)
//   sparse family -> nw.tileHrowMat / tileHcolMat, the geometry fields NwTrace2_Sparse reads
//                    (run_types.hpp:97-100, set as gpu9 does at :696-699), res.align_cost
//                    (= the last-tile recompute, nwalign_gpu9_mlsp_diagdiagdiag.cu:713-716)
// and res.sw_align through the reference's own Stopwatch: res.sw_align.start() here, then
// libgsa calls Stopwatch::lap at each phase boundary (gsa_set_lap_callback), with the
// reference's lap names align.alloc / cpy_dev / init_hdr / calc / cpy_host
// (stopwatch.cpp:43-50, file_formats.cpp:505-519).  Status codes have NwStat's numbering.
//
// Differences against the reference's types, the only edits when this file moves into the
// reference's src/ (INTEGRATION.md lists them): the include below becomes "run_types.hpp" +
// "gsa.h"; the result buffers are HostArray<int> (init(n) in place of resize(n)); res.hipStat
// is res.cudaStat; update_peak_mem is the reference's updateNwAlgPeakMemUsage; nw.ctx (the
// mirror's device context) is a per-process gsa_ctx created where initNwInput sets the device up.
#include <algorithm>
#include <exception>

#include "nw_host.hpp"

namespace gsa_host {

namespace {

// libgsa -> Stopwatch::lap of the result being filled (src/stopwatch.hpp:19)
void onLap(void* sw, const char* lapName) { static_cast<Stopwatch*>(sw)->lap(lapName); }

// Starts res.sw_align and routes the context's phase boundaries into it for one call.
struct LapScope
{
    gsa_ctx* ctx;
    LapScope(gsa_ctx* c, Stopwatch& sw) : ctx(c)
    {
        sw.start();
        gsa_set_lap_callback(ctx, onLap, &sw);
    }
    ~LapScope() { gsa_set_lap_callback(ctx, nullptr, nullptr); }
};

NwStat checkInput(const NwAlgInput& nw)
{
    if (!nw.ctx || nw.adjrows < 1 || nw.adjcols < 1 || (int)nw.seqY.size() != nw.adjrows ||
        (int)nw.seqX.size() != nw.adjcols || (int)nw.subst.size() != nw.substsz * nw.substsz)
        return NwStat::errorInvalidValue;
    return NwStat::success;
}

// Peak-alloc columns from the context's launch footprints (updateNwAlgPeakMemUsage,
// nwalign_shared.cpp:5-25): kernel attributes x resident workgroups of every fill of the call.
void update_peak_mem(const NwAlgInput& nw, NwAlgResult& res)
{
    gsa_mem_stats m {};
    if (gsa_mem_stats_get(nw.ctx, &m) != GSA_SUCCESS) return;
    res.globalMemPeakAllocs = std::max(res.globalMemPeakAllocs, (size_t)m.glmem_peak_allocs);
    res.sharedMemPeakAllocs = std::max(res.sharedMemPeakAllocs, (size_t)m.shmem_peak_allocs);
    res.localMemPeakAllocs = std::max(res.localMemPeakAllocs, (size_t)m.locmem_peak_allocs);
    res.regMemPeakAllocs = std::max(res.regMemPeakAllocs, (size_t)m.regmem_peak_allocs);
}

// The sparse family's tile: width from the slot's parameters, height the engine's (1024).
NwStat alignMlsp(int tileBx, NwAlgInput& nw, NwAlgResult& res, bool overlap)
{
    if (NwStat s = checkInput(nw); s != NwStat::success) return s;
    gsa_sparse_geom g {};
    if (int st = gsa_sparse_geometry(nw.adjrows, nw.adjcols, tileBx, &g); st != GSA_SUCCESS) return (NwStat)st;
    int cost = 0;
    int st;
    {
        // the stopwatch starts before the host result arrays are allocated, so that their
        // allocation is part of align.alloc (nwalign_gpu9_mlsp_diagdiagdiag.cu:434-459)
        LapScope laps(nw.ctx, res.sw_align);
        try
        {
            nw.tileHrowMat.resize((size_t)g.hrowElems);
            nw.tileHcolMat.resize((size_t)g.hcolElems);
        }
        catch (const std::exception&)
        {
            return NwStat::errorMemoryAllocation;
        }
        gsa_mem_stats_reset(nw.ctx);  // peaks of this call only (res keeps the max over runs)
        st = (overlap ? gsa_align_sparse_pt : gsa_align_sparse)(nw.ctx, nw.seqY.data(), nw.adjrows, nw.seqX.data(),
                                                                nw.adjcols, nw.subst.data(), nw.substsz, nw.gapoCost,
                                                                tileBx, nw.tileHrowMat.data(), nw.tileHcolMat.data(),
                                                                &g, &cost, nullptr);
    }
    res.hipStat = gsa_last_hip_error(nw.ctx);  // the raw runtime error, as res.cudaStat keeps it
    if (st != GSA_SUCCESS) return (NwStat)st;  // same numbering as NwStat
    nw.geom = g;
    nw.tileHdrMatRows = g.tileHdrMatRows;
    nw.tileHdrMatCols = g.tileHdrMatCols;
    nw.tileHrowLen = g.tileHrowLen;
    nw.tileHcolLen = g.tileHcolLen;
    res.align_cost = cost;
    res.globalMemPeakAllocs =
        std::max(res.globalMemPeakAllocs, (nw.tileHrowMat.size() + nw.tileHcolMat.size()) * sizeof(int));
    update_peak_mem(nw, res);
    return NwStat::success;
}

// Plain family: the full (adjrows x adjcols) matrix in nw.score.  The wavefront geometry is the
// engine's; the slots' tiling parameters are checked (slotGeometry) and noted.
NwStat alignFull(NwAlgInput& nw, NwAlgResult& res)
{
    if (NwStat s = checkInput(nw); s != NwStat::success) return s;
    int cost = 0;
    int st;
    {
        LapScope laps(nw.ctx, res.sw_align);  // host allocation inside align.alloc, as the reference's
        try
        {
            nw.score.resize((size_t)nw.adjrows * (size_t)nw.adjcols);
        }
        catch (const std::exception&)
        {
            return NwStat::errorMemoryAllocation;
        }
        gsa_mem_stats_reset(nw.ctx);
        st = gsa_align_full(nw.ctx, nw.seqY.data(), nw.adjrows, nw.seqX.data(), nw.adjcols, nw.subst.data(),
                            nw.substsz, nw.gapoCost, nw.score.data(), &cost, nullptr);
    }
    res.hipStat = gsa_last_hip_error(nw.ctx);
    if (st != GSA_SUCCESS) return (NwStat)st;
    res.align_cost = cost;
    res.globalMemPeakAllocs = std::max(res.globalMemPeakAllocs, nw.score.size() * sizeof(int));
    update_peak_mem(nw, res);
    return NwStat::success;
}

// The slot's parameters -> the engine geometry that runs, noted in the TSV's alg_params column
// (engine_tileBx / engine_tileBy) so a row says which tile the headers have.
NwStat runSlot(const char* slot, const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res, bool overlap)
{
    SlotGeometry geo;
    if (NwStat s = slotGeometry(slot, pr, geo); s != NwStat::success) return s;
    if (geo.sparse)
    {
        std::string& j = res.algParamsJson;
        const std::string note = "\"engine_tileBx\":" + std::to_string(geo.tileBx) +
                                 ",\"engine_tileBy\":" + std::to_string(gsa_sparse_tile_by());
        if (j.size() >= 2 && j.back() == '}' && j.find("engine_tileBx") == std::string::npos)
            j.insert(j.size() - 1, (j.size() > 2 ? "," : "") + note);
        return alignMlsp(geo.tileBx, nw, res, overlap);
    }
    return alignFull(nw, res);
}

}  // namespace

// ---- the parameter contract of the reference's slots ---------------------------------------
// Each reference slot reads its own parameters with pr.at() inside a try block, so a parameter
// the file does not list throws and the slot returns errorInvalidValue, and so does a value its
// rules reject (nwalign_gpu1_ml_diag.cu:82-93, gpu2:125-141, gpu3:297-311, gpu4:292-310,
// gpu5:322-333, gpu6:303-321, gpu7_mlsp:305-320, gpu8:325-340, gpu9:382-414).  Both are kept
// for the Gpu1..9 names: every parameter the reference slot reads is required.  The rules use
// the reference's units: a warp is kParamWarp = 32 threads (the unit its parameter files are
// tuned in, param_best.json:1, an RTX 3090), a block at most 1024 threads.  This engine's own
// NwAlign_Amd_Strip_* slots have defaults (tileBx 256) and need no parameter.
// The sparse slots' tile width maps to the engine's nearest (a multiple of 16, >= 64):
//   gpu7/gpu8: tileBx;
//   gpu9: the reference's derived width, tileBx = k*subtileBx - (tileBy - 1) with tileBy =
//         subtileRows*32 and k = ceil((subtileCols*subtileBx + tileBy - 1) / subtileBx) (:389-398);
//   this engine's slots: tileBx itself, which must then be a multiple of 16 and >= 64.
// The tile height is the engine's 1024 whatever the slot asks (gsa_sparse_tile_by).
NwStat slotGeometry(const std::string& slot, const NwAlgParams& pr, SlotGeometry& out)
{
    constexpr int kParamWarp = 32, kMaxThreads = 1024;
    // pr.at() throws std::out_of_range for a missing name, caught below as the reference does
    const auto req = [&](const char* n) { return (long long)pr.at(n).curr(); };
    const auto threads = [&](const char* n) {
        const long long v = req(n);
        return v >= kParamWarp && v <= kMaxThreads;
    };
    const auto atLeast1 = [&](const char* n) { return req(n) >= 1; };
    const auto warpMultiple = [&](const char* n) {
        const long long v = req(n);
        return v >= 1 && v % kParamWarp == 0;
    };
    const auto nearest16 = [](long long w) { return (int)std::max<long long>(64, ((w + 8) / 16) * 16); };
    out = SlotGeometry {};
    const auto bad = NwStat::errorInvalidValue;
    try
    {
        if (slot == "NwAlign_Gpu1_Ml_Diag") return threads("threadsPerBlock") ? NwStat::success : bad;
        if (slot == "NwAlign_Gpu2_Ml_DiagRow2Pass")
        {
            const bool ok = atLeast1("tileBx") && atLeast1("tileBy");
            return ok && threads("threadsPerBlock") ? NwStat::success : bad;
        }
        if (slot == "NwAlign_Gpu3_Ml_DiagDiag")
        {
            const bool ok = threads("threadsPerBlockA");
            return ok && atLeast1("tileBx") ? NwStat::success : bad;
        }
        if (slot == "NwAlign_Gpu4_Ml_DiagDiag2Pass" || slot == "NwAlign_Gpu6_Coop_DiagDiag2Pass")
        {
            // all three are read before any is checked (gpu4:294-296)
            const long long ax = req("tileAx"), ay = req("tileAy"), bx = req("tileBx");
            return ax >= 1 && ay >= 1 && bx >= 1 && warpMultiple("tileAx") ? NwStat::success : bad;
        }
        if (slot == "NwAlign_Gpu5_Coop_DiagDiag") return atLeast1("tileAx") ? NwStat::success : bad;
        if (slot == "NwAlign_Amd_Strip_Full") return NwStat::success;
        out.sparse = true;
        if (slot == "NwAlign_Gpu7_Mlsp_DiagDiag" || slot == "NwAlign_Gpu8_Mlsp_DiagDiag")
        {
            const long long tpb = req("threadsPerBlockA"), bx = req("tileBx"), wdf = req("warpDivFactorB");
            if (tpb < kParamWarp || tpb > kMaxThreads || bx < 1 || wdf < 1) return bad;
            out.tileBx = nearest16(bx);
            return NwStat::success;
        }
        if (slot == "NwAlign_Gpu9_Mlsp_DiagDiagDiag")
        {
            const long long tpb = req("threadsPerBlockA"), rows = req("subtileRows"), cols = req("subtileCols");
            const long long sbx = req("subtileBx");
            if (rows < 1 || cols < 1 || sbx < 1 || tpb < kParamWarp || tpb > kMaxThreads) return bad;
            const long long tileBy = rows * kParamWarp;
            const long long k = (cols * sbx + tileBy - 1 + sbx - 1) / sbx;
            const long long tileBx = k * sbx - (tileBy - 1);
            if (sbx < kParamWarp || tileBx < tileBy) return bad;
            out.tileBx = nearest16(tileBx);
            return NwStat::success;
        }
        if (slot != "NwAlign_Amd_Strip_Mlsp" && slot != "NwAlign_Amd_Strip_Mlsppt") return bad;
        int v = 256;
        if (pr.has("tileBx"))
        {
            v = pr.at("tileBx").curr();
            if (v < 64 || v % 16 != 0) return bad;
        }
        out.tileBx = v;
        return NwStat::success;
    }
    catch (const std::exception&)
    {
        return bad;  // as the reference's try / catch around pr.at()
    }
}

// One adapter per slot name (NwAlignFn has no name argument): the reference's Gpu1..9 slots with
// their parameter rules, and this engine's own three names.
#define GSA_SLOT(name, overlap) \
    NwStat name(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res) { return runSlot(#name, pr, nw, res, overlap); }
GSA_SLOT(NwAlign_Gpu1_Ml_Diag, false)
GSA_SLOT(NwAlign_Gpu2_Ml_DiagRow2Pass, false)
GSA_SLOT(NwAlign_Gpu3_Ml_DiagDiag, false)
GSA_SLOT(NwAlign_Gpu4_Ml_DiagDiag2Pass, false)
GSA_SLOT(NwAlign_Gpu5_Coop_DiagDiag, false)
GSA_SLOT(NwAlign_Gpu6_Coop_DiagDiag2Pass, false)
GSA_SLOT(NwAlign_Gpu7_Mlsp_DiagDiag, false)
GSA_SLOT(NwAlign_Gpu8_Mlsp_DiagDiag, false)
GSA_SLOT(NwAlign_Gpu9_Mlsp_DiagDiagDiag, false)
GSA_SLOT(NwAlign_Amd_Strip_Full, false)
GSA_SLOT(NwAlign_Amd_Strip_Mlsp, false)
// mlsppt ("multi-launch sparse with parallel transfer", README.md:39 of the reference, never
// implemented there): the same outputs, the header copy-back overlapped with the fill.
GSA_SLOT(NwAlign_Amd_Strip_Mlsppt, true)
#undef GSA_SLOT

}  // namespace gsa_host
