// CPU check of the NwAlignFn adapters (gpuseqalign_amd/host/nwalign_amd.cpp): compiled against the
// host mirror of the reference's types, linked with libgsa.so, run without a GPU.  It checks the
// adapters' contract that needs no device: the registry slots point at them, a missing device
// context is errorInvalidValue (no exception crosses), and Stopwatch::lap accumulates per name as
// the reference's does (stopwatch.cpp:43-50), which is what gsa_set_lap_callback drives.
#include <cstdio>
#include <map>
#include <thread>

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
