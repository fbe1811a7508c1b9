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

// Sparse family: tile header matrices.  Parameter "tileBx" (a multiple of 16, >= 64) selects the
// tile width, default 256; the tile height is the engine's (gsa_sparse_tile_by()).
NwStat alignMlsp(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res, bool overlap)
{
    if (NwStat s = checkInput(nw); s != NwStat::success) return s;
    int tileBx = 256;
    if (pr.has("tileBx"))
    {
        const int v = pr.at("tileBx").curr();
        if (v >= 64 && v % 16 == 0) tileBx = v;
    }
    gsa_sparse_geom g {};
    if (int st = gsa_sparse_geometry(nw.adjrows, nw.adjcols, tileBx, &g); st != GSA_SUCCESS) return (NwStat)st;
    try
    {
        nw.tileHrowMat.resize((size_t)g.hrowElems);
        nw.tileHcolMat.resize((size_t)g.hcolElems);
    }
    catch (const std::exception&)
    {
        return NwStat::errorMemoryAllocation;
    }
    int cost = 0;
    gsa_mem_stats_reset(nw.ctx);  // peaks of this call only (res keeps the max over runs)
    int st;
    {
        LapScope laps(nw.ctx, res.sw_align);
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

}  // namespace

// Plain family (the NwAlign_Gpu1..6 slots): the full (adjrows x adjcols) matrix in nw.score.  No
// tunables: the wavefront geometry is fixed by the hardware; parameters the
// reference's files list for these slots are accepted and ignored.
NwStat NwAlign_Amd_Strip_Full(const NwAlgParams&, NwAlgInput& nw, NwAlgResult& res)
{
    if (NwStat s = checkInput(nw); s != NwStat::success) return s;
    try
    {
        nw.score.resize((size_t)nw.adjrows * (size_t)nw.adjcols);
    }
    catch (const std::exception&)
    {
        return NwStat::errorMemoryAllocation;
    }
    int cost = 0;
    gsa_mem_stats_reset(nw.ctx);
    int st;
    {
        LapScope laps(nw.ctx, res.sw_align);
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

// Sparse family (the NwAlign_Gpu7..9 slots).
NwStat NwAlign_Amd_Strip_Mlsp(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res)
{
    return alignMlsp(pr, nw, res, false);
}

// mlsppt ("multi-launch sparse with parallel transfer", README.md:39 of the reference, never
// implemented there): the same outputs, the header copy-back overlapped with the fill.
NwStat NwAlign_Amd_Strip_Mlsppt(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res)
{
    return alignMlsp(pr, nw, res, true);
}

}  // namespace gsa_host
