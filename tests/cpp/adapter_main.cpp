// CPU check of the NwAlignFn adapters (gpuseqalign_amd/host/nwalign_amd.cpp): compiled against the
// host mirror of the reference's types, linked with libgsa.so, run without a GPU.  It checks the
// adapters' contract that needs no device: the registry slots point at them, a missing device
// context is errorInvalidValue (no exception crosses), and Stopwatch::lap accumulates per name as
// the reference's does (stopwatch.cpp:43-50), which is what gsa_set_lap_callback drives.
#include <cstdio>
#include <map>
#include <thread>
#include <vector>

#include "nw_host.hpp"

using namespace gsa_host;

int main()
{
    int bad = 0;
    std::map<std::string, NwAlgorithm> m;
    getNwAlgorithmMap(m);
    for (const char* n : {"NwAlign_Gpu3_Ml_DiagDiag", "NwAlign_Gpu9_Mlsp_DiagDiagDiag", "NwAlign_Amd_Strip_Mlsppt"})
        if (!m.count(n)) { std::printf("missing slot %s\n", n); ++bad; }
    NwAlgParams pr;
    NwAlgInput nw;  // no device context
    nw.adjrows = nw.adjcols = 1;
    nw.seqY = nw.seqX = {0};
    nw.substsz = 1;
    nw.subst = {1};
    for (auto fn : {NwAlign_Amd_Strip_Full, NwAlign_Amd_Strip_Mlsp, NwAlign_Amd_Strip_Mlsppt})
    {
        NwAlgResult res;
        if (fn(pr, nw, res) != NwStat::errorInvalidValue) { std::printf("no-context call not rejected\n"); ++bad; }
        if (!res.sw_align.laps.empty()) { std::printf("laps recorded for a rejected call\n"); ++bad; }
    }
    // the slots' parameter contract: every entry of the reference's param_best.json is accepted, with
    // the engine tile the sparse slots map to; values the reference's functions reject are
    // errorInvalidValue (nwalign_gpu9_mlsp_diagdiagdiag.cu:382-414 and the other slots' checks)
    auto params = [](std::initializer_list<std::pair<const char*, int>> kv) {
        NwAlgParams p;
        for (auto& [k, v] : kv) p.params.push_back({k, NwAlgParam {{v}, 0}});
        return p;
    };
    struct Case
    {
        const char* slot;
        NwAlgParams pr;
        NwStat want;
        int tileBx;  // sparse slots: the engine width that runs (0: plain)
    };
    const Case cases[] = {
        // resrc/param_best.json
        {"NwAlign_Gpu1_Ml_Diag", params({{"threadsPerBlock", 64}}), NwStat::success, 0},
        {"NwAlign_Gpu2_Ml_DiagRow2Pass", params({{"tileBx", 8}, {"tileBy", 4}, {"threadsPerBlock", 64}}), NwStat::success, 0},
        {"NwAlign_Gpu3_Ml_DiagDiag", params({{"threadsPerBlockA", 96}, {"tileBx", 54}}), NwStat::success, 0},
        {"NwAlign_Gpu4_Ml_DiagDiag2Pass", params({{"tileAx", 384}, {"tileAy", 32}, {"tileBx", 52}}), NwStat::success, 0},
        {"NwAlign_Gpu5_Coop_DiagDiag", params({{"tileAx", 52}}), NwStat::success, 0},
        {"NwAlign_Gpu6_Coop_DiagDiag2Pass", params({{"tileAx", 192}, {"tileAy", 128}, {"tileBx", 66}}), NwStat::success, 0},
        {"NwAlign_Gpu7_Mlsp_DiagDiag", params({{"threadsPerBlockA", 96}, {"tileBx", 70}, {"warpDivFactorB", 1}}), NwStat::success, 64},
        {"NwAlign_Gpu8_Mlsp_DiagDiag", params({{"threadsPerBlockA", 160}, {"tileBx", 76}, {"warpDivFactorB", 1}}), NwStat::success, 80},
        {"NwAlign_Gpu9_Mlsp_DiagDiagDiag", params({{"threadsPerBlockA", 128}, {"subtileRows", 4}, {"subtileCols", 4}, {"subtileBx", 48}}), NwStat::success, 208},
        // this engine's own slots: tileBx with a default of 256
        {"NwAlign_Amd_Strip_Mlsp", params({{"tileBx", 512}}), NwStat::success, 512},
        {"NwAlign_Amd_Strip_Mlsp", params({}), NwStat::success, 256},
        {"NwAlign_Amd_Strip_Mlsppt", params({{"tileBx", 128}}), NwStat::success, 128},
        {"NwAlign_Amd_Strip_Full", params({}), NwStat::success, 0},
        // rejected as the reference rejects them
        {"NwAlign_Amd_Strip_Mlsp", params({{"tileBx", 100}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Amd_Strip_Mlsppt", params({{"tileBx", 48}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu9_Mlsp_DiagDiagDiag", params({{"threadsPerBlockA", 128}, {"subtileRows", 4}, {"subtileCols", 4}, {"subtileBx", 16}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu9_Mlsp_DiagDiagDiag", params({{"threadsPerBlockA", 2048}, {"subtileRows", 1}, {"subtileCols", 1}, {"subtileBx", 64}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu7_Mlsp_DiagDiag", params({{"threadsPerBlockA", 96}, {"tileBx", 0}, {"warpDivFactorB", 1}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu8_Mlsp_DiagDiag", params({{"threadsPerBlockA", 16}, {"tileBx", 76}, {"warpDivFactorB", 1}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu4_Ml_DiagDiag2Pass", params({{"tileAx", 100}, {"tileAy", 32}, {"tileBx", 52}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu1_Ml_Diag", params({{"threadsPerBlock", 2000}}), NwStat::errorInvalidValue, 0},
        {"NwAlign_Gpu5_Coop_DiagDiag", params({{"tileAx", -1}}), NwStat::errorInvalidValue, 0},
    };
    // a parameter the reference slot reads with pr.at() and the file does not list: the slot throws
    // and returns errorInvalidValue (nwalign_gpu9_mlsp_diagdiagdiag.cu:384-387,411-414, gpu3:299-300,
    // gpu7:307-309, gpu8:327-329 and the others); every required name is dropped in turn from the
    // slot's param_best.json entry
    std::vector<Case> all(std::begin(cases), std::end(cases));
    const std::vector<std::pair<const char*, std::vector<std::pair<const char*, int>>>> best = {
        {"NwAlign_Gpu1_Ml_Diag", {{"threadsPerBlock", 64}}},
        {"NwAlign_Gpu2_Ml_DiagRow2Pass", {{"tileBx", 8}, {"tileBy", 4}, {"threadsPerBlock", 64}}},
        {"NwAlign_Gpu3_Ml_DiagDiag", {{"threadsPerBlockA", 96}, {"tileBx", 54}}},
        {"NwAlign_Gpu4_Ml_DiagDiag2Pass", {{"tileAx", 384}, {"tileAy", 32}, {"tileBx", 52}}},
        {"NwAlign_Gpu5_Coop_DiagDiag", {{"tileAx", 52}}},
        {"NwAlign_Gpu6_Coop_DiagDiag2Pass", {{"tileAx", 192}, {"tileAy", 128}, {"tileBx", 66}}},
        {"NwAlign_Gpu7_Mlsp_DiagDiag", {{"threadsPerBlockA", 96}, {"tileBx", 70}, {"warpDivFactorB", 1}}},
        {"NwAlign_Gpu8_Mlsp_DiagDiag", {{"threadsPerBlockA", 160}, {"tileBx", 76}, {"warpDivFactorB", 1}}},
        {"NwAlign_Gpu9_Mlsp_DiagDiagDiag", {{"threadsPerBlockA", 128}, {"subtileRows", 4}, {"subtileCols", 4}, {"subtileBx", 48}}},
    };
    int missingCases = 0;
    for (const auto& [slot, kv] : best)
    {
        all.push_back({slot, params({}), NwStat::errorInvalidValue, 0});
        for (size_t drop = 0; drop < kv.size(); ++drop)
        {
            NwAlgParams p;
            for (size_t i = 0; i < kv.size(); ++i)
                if (i != drop) p.params.push_back({kv[i].first, NwAlgParam {{kv[i].second}, 0}});
            all.push_back({slot, p, NwStat::errorInvalidValue, 0});
            ++missingCases;
        }
    }
    if (missingCases != 23) { std::printf("missing-parameter cases: %d, want 23\n", missingCases); ++bad; }
    for (const Case& c : all)
    {
        SlotGeometry geo;
        const NwStat st = slotGeometry(c.slot, c.pr, geo);
        if (st != c.want || (st == NwStat::success && geo.tileBx != c.tileBx))
        {
            std::printf("slot %s %s: stat %d tileBx %d, want %d %d\n", c.slot, c.pr.toJson().c_str(), (int)st,
                        geo.tileBx, (int)c.want, c.tileBx);
            ++bad;
        }
        // through the registry slot (no device: a rejected parameter wins, an accepted one reaches
        // the input check)
        NwAlgResult res;
        res.algParamsJson = c.pr.toJson();
        NwAlgInput in = nw;
        const NwStat s2 = m.at(c.slot).align(c.pr, in, res);
        if (s2 != NwStat::errorInvalidValue) { std::printf("slot %s without a device: %d\n", c.slot, (int)s2); ++bad; }
        if (c.tileBx && res.algParamsJson.find("\"engine_tileBx\":" + std::to_string(c.tileBx)) == std::string::npos)
        {
            std::printf("slot %s: alg_params %s lacks the engine tile\n", c.slot, res.algParamsJson.c_str());
            ++bad;
        }
    }
    // the callback route: what libgsa calls at each boundary, into a Stopwatch
    gsa_lap_fn fn = [](void* sw, const char* name) { static_cast<Stopwatch*>(sw)->lap(name); };
    Stopwatch sw;
    sw.start();
    std::this_thread::sleep_for(std::chrono::milliseconds(3));
    fn(&sw, "align.calc");
    fn(&sw, "align.cpy_host");
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    fn(&sw, "align.calc");
    const float calc = sw.get_or_default("align.calc"), host = sw.get_or_default("align.cpy_host");
    if (sw.laps.size() != 2 || calc < 4.5f || host > 1.0f) { std::printf("lap semantics: calc %.3f host %.3f\n", calc, host); ++bad; }
    std::printf("adapter check: %s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
