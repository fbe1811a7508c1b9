// nw_main.cpp -- `gsa_nw`, the command-line bench driver of the MI355X engine.
//
// Same flags, defaults, loop order and verification as the reference's `nw` driver
// (src/cmd_parser.cpp:123-300, src/benchmark.cpp:120-147 and :393-520):
//   for each algorithm (the reference algorithm first)
//     for each sequence pair
//       for each parameter combination
//         warmup runs (discarded when successful), then sample runs:
//           align -> [hash] -> [trace] -> verify {align_cost, score_hash, trace_hash}
//           against the first algorithm that aligned the same pair
//         one TSV line per combination (laps averaged over the sample runs)
// The device work is libgsa.so (include/gsa.h) behind the NwAlgorithm table (nw_host.hpp).
#include <chrono>
#include <cstdlib>
#include <ctime>
#include <fstream>
#include <iostream>
#include <map>
#include <optional>
#include <string>
#include <sys/stat.h>
#include <tuple>
#include <vector>

#include "nw_host.hpp"

using namespace gsa_host;

namespace {

struct CmdArgs
{
    std::string substPath = "./resrc/subst.json";
    std::string algParamPath, seqPath, seqPairPath, resPath, debugPath;
    std::string substName = "blosum62";
    int gapoCost = -11, gapeCost = 0;
    std::vector<std::string> algNames;
    std::string refAlgName;
    int warmupPerAlign = 0, samplesPerAlign = 1;
    bool fCalcTrace = false, fCalcScoreHash = false, fWriteProgress = false, fPrintScore = false, fPrintTrace = false;
    int device = 0;
    bool dryRun = false;
};

void usage(std::ostream& os)
{
    os << "gsa_nw --algParamPath \"path\" --seqPath \"path\" [params]\n"
          "\n"
          "Parameters (same as the GpuSeqAlign `nw` driver):\n"
          "-b, --substPath <path>     JSON substitution matrices, default \"./resrc/subst.json\".\n"
          "-r, --algParamPath <path>  JSON algorithm parameters.\n"
          "-s, --seqPath <path>       FASTA sequences.\n"
          "-p, --seqPairPath <path>   Sequence pairs \"seqY[l:r] seqX[l:r]\" per line; default: every sequence\n"
          "                           against the first one.\n"
          "-o, --resPath <path>       TSV results, default \"./logs/<datetime>.tsv\".\n"
          "--substName <name>         Substitution matrix, default \"blosum62\".\n"
          "--gapoCost <cost>          Gap open (linear gap) cost, default -11.\n"
          "--gapeCost <cost>          Unused, default 0.\n"
          "--algName <name>           Algorithm to run (repeatable); default: all in the parameter file.\n"
          "--refAlgName <name>        Source-of-truth algorithm, run first; default: the first algorithm.\n"
          "--warmupPerAlign <num>     Warmup runs per alignment, default 0.\n"
          "--samplesPerAlign <num>    Measured runs per alignment, default 1.\n"
          "--fCalcTrace               Compute the traceback.\n"
          "--fCalcScoreHash           Compute the score hash.\n"
          "--fWriteProgress           Print progress on stdout.\n"
          "--debugPath <path>         Where --fPrintScore/--fPrintTrace write, default \"./logs/<datetime>_debug.txt\".\n"
          "--fPrintScore              Print score matrices / tile headers.\n"
          "--fPrintTrace              Print traces.\n"
          "--device <id>              HIP device (this engine's addition), default 0.\n"
          "--dryRun                   Read and check every input, print the run plan, touch no device.\n"
          "-h, --help                 Print help and exit.\n";
}

std::string iso_datetime()
{
    std::time_t t = std::time(nullptr);
    char buf[64];
    std::strftime(buf, sizeof buf, "%Y%m%d_%H%M%S", std::localtime(&t));
    return buf;
}

NwStat parse_args(int argc, const char* argv[], CmdArgs& a)
{
    if (argc == 1)
    {
        usage(std::cout);
        std::cerr << "error: expected command parameters\n";
        return NwStat::errorInvalidValue;
    }
    auto take = [&](int& i, std::string& dst, const std::string& name) {
        if (i + 1 >= argc)
        {
            std::cerr << "error: expected value after parameter \"" << name << "\"\n";
            return false;
        }
        dst = argv[++i];
        return true;
    };
    auto take_int = [&](int& i, int& dst, const std::string& name, bool nonneg) {
        std::string v;
        if (!take(i, v, name)) return false;
        try
        {
            size_t used = 0;
            dst = std::stoi(v, &used);
            if (used != v.size() || (nonneg && dst < 0)) throw std::invalid_argument(v);
        }
        catch (const std::exception&)
        {
            std::cerr << "error: invalid value for \"" << name << "\": \"" << v << "\"\n";
            return false;
        }
        return true;
    };
    bool print_flags_given = false;
    for (int i = 1; i < argc; ++i)
    {
        std::string s = argv[i];
        bool ok = true;
        if (s == "-b" || s == "--substPath") ok = take(i, a.substPath, s);
        else if (s == "-r" || s == "--algParamPath") ok = take(i, a.algParamPath, s);
        else if (s == "-s" || s == "--seqPath") ok = take(i, a.seqPath, s);
        else if (s == "-p" || s == "--seqPairPath") ok = take(i, a.seqPairPath, s);
        else if (s == "-o" || s == "--resPath") ok = take(i, a.resPath, s);
        else if (s == "--substName") ok = take(i, a.substName, s);
        else if (s == "--gapoCost") ok = take_int(i, a.gapoCost, s, false);
        else if (s == "--gapeCost") ok = take_int(i, a.gapeCost, s, false);
        else if (s == "--algName")
        {
            std::string v;
            ok = take(i, v, s);
            if (ok) a.algNames.push_back(v);
        }
        else if (s == "--refAlgName") ok = take(i, a.refAlgName, s);
        else if (s == "--warmupPerAlign") ok = take_int(i, a.warmupPerAlign, s, true);
        else if (s == "--samplesPerAlign") ok = take_int(i, a.samplesPerAlign, s, true);
        else if (s == "--fCalcTrace") a.fCalcTrace = true;
        else if (s == "--fCalcScoreHash") a.fCalcScoreHash = true;
        else if (s == "--fWriteProgress") a.fWriteProgress = true;
        else if (s == "--debugPath") ok = take(i, a.debugPath, s);
        else if (s == "--fPrintScore") a.fPrintScore = print_flags_given = true;
        else if (s == "--fPrintTrace") a.fPrintTrace = print_flags_given = true;
        else if (s == "--device") ok = take_int(i, a.device, s, true);
        else if (s == "--dryRun") a.dryRun = true;
        else if (s == "-h" || s == "--help")
        {
            usage(std::cout);
            return NwStat::helpMenuRequested;
        }
        else
        {
            usage(std::cout);
            std::cerr << "error: unknown parameter: \"" << s << "\"\n";
            return NwStat::errorInvalidValue;
        }
        if (!ok) return NwStat::errorInvalidValue;
    }
    if (a.algParamPath.empty())
    {
        std::cerr << "error: expected parameter: \"--algParamPath\"\n";
        return NwStat::errorInvalidValue;
    }
    if (a.seqPath.empty())
    {
        std::cerr << "error: expected parameter: \"--seqPath\"\n";
        return NwStat::errorInvalidValue;
    }
    const std::string dt = iso_datetime();
    if (a.resPath.empty()) a.resPath = "./logs/" + dt + ".tsv";
    if (print_flags_given && a.debugPath.empty()) a.debugPath = "./logs/" + dt + "_debug.txt";
    return NwStat::success;
}

NwStat open_out(const std::string& path, std::ofstream& ofs)
{
    size_t slash = path.find_last_of('/');
    if (slash != std::string::npos && slash > 0)
    {
        std::string dir = path.substr(0, slash);
        std::string cur;
        for (size_t k = 0; k <= dir.size(); ++k)
            if (k == dir.size() || dir[k] == '/')
            {
                cur = dir.substr(0, k);
                if (!cur.empty()) mkdir(cur.c_str(), 0755);
            }
    }
    ofs.open(path);
    return ofs ? NwStat::success : NwStat::errorIoStream;
}

struct CompareKey
{
    std::string y, x;
    int64_t yl, yr, xl, xr;
    bool operator<(const CompareKey& o) const
    {
        return std::tie(y, x, yl, yr, xl, xr) < std::tie(o.y, o.x, o.yl, o.yr, o.xl, o.xr);
    }
};

}  // namespace

int main(int argc, const char* argv[])
{
    CmdArgs a;
    if (NwStat s = parse_args(argc, argv, a); s != NwStat::success) return s == NwStat::helpMenuRequested ? 0 : (int)s;

    std::string err;
    NwSubstData substData;
    NwAlgParamsData paramData;
    std::vector<NwSeq> seqs;
    std::vector<NwSeqPair> pairs;
    if (readSubstFile(a.substPath, substData, err) != NwStat::success ||
        readAlgParamsFile(a.algParamPath, paramData, err) != NwStat::success ||
        readFastaFile(a.seqPath, substData, seqs, err) != NwStat::success)
    {
        std::cerr << "error: " << err << "\n";
        return (int)NwStat::errorInvalidFormat;
    }
    if (!a.seqPairPath.empty())
    {
        if (readSeqPairFile(a.seqPairPath, seqs, pairs, err) != NwStat::success)
        {
            std::cerr << "error: " << err << "\n";
            return (int)NwStat::errorInvalidFormat;
        }
    }
    else
    {
        for (size_t k = 1; k < seqs.size(); ++k)
        {
            NwSeqPair p;
            p.seqY_id = seqs[k].id;
            p.seqX_id = seqs[0].id;
            p.seqY_range = NwRange {false, false, 0, (int64_t)seqs[k].seq.size() - 1};
            p.seqX_range = NwRange {false, false, 0, (int64_t)seqs[0].seq.size() - 1};
            pairs.push_back(p);
        }
        if (pairs.empty())
        {
            std::cerr << "error: since seqPairPath is empty, at least two sequences are necessary for default alignment\n";
            return (int)NwStat::errorInvalidFormat;
        }
    }

    NwAlgInput nw;
    bool subst_found = false;
    for (auto& kv : substData.substMap)
        if (kv.first == a.substName)
        {
            nw.subst = kv.second;
            subst_found = true;
        }
    if (!subst_found)
    {
        std::cerr << "error: unknown substitution matrix: \"" << a.substName << "\"\n";
        return (int)NwStat::errorInvalidValue;
    }
    nw.substsz = (int)substData.letterMap.size();
    nw.gapoCost = a.gapoCost;

    std::map<std::string, NwAlgorithm> algMap;
    getNwAlgorithmMap(algMap);
    std::vector<std::string> algNames = a.algNames;
    if (algNames.empty())
        for (auto& kv : paramData.paramMap) algNames.push_back(kv.first);
    // algorithms of the reference that are not part of this engine (its CPU oracle family)
    std::vector<std::string> run;
    for (auto& n : algNames)
    {
        bool in_params = false;
        for (auto& kv : paramData.paramMap) in_params |= kv.first == n;
        if (!in_params)
        {
            std::cerr << "error: algorithm \"" << n << "\" has no entry in the parameter file\n";
            return (int)NwStat::errorInvalidValue;
        }
        if (!algMap.count(n))
        {
            std::cerr << "warning: algorithm \"" << n << "\" is not provided by this engine, skipped\n";
            continue;
        }
        run.push_back(n);
    }
    if (run.empty())
    {
        std::cerr << "error: no runnable algorithm selected\n";
        return (int)NwStat::errorInvalidValue;
    }
    std::string refAlg = a.refAlgName.empty() ? run.front() : a.refAlgName;
    for (size_t k = 0; k < run.size(); ++k)
        if (run[k] == refAlg)
        {
            run.erase(run.begin() + (long)k);
            run.insert(run.begin(), refAlg);
            break;
        }

    if (a.dryRun)
    {
        std::cout << "subst " << a.substName << " substsz " << nw.substsz << " gapo " << a.gapoCost << "\n";
        for (auto& n : run)
        {
            NwAlgParams params;
            for (auto& kv : paramData.paramMap)
                if (kv.first == n) params = kv.second;
            int combos = 0;
            for (params.reset(); params.hasCurr(); params.next()) ++combos;
            std::cout << "alg " << n << " combos " << combos << "\n";
        }
        for (auto& p : pairs)
        {
            const NwSeq *y = nullptr, *x = nullptr;
            for (auto& q : seqs)
            {
                if (q.id == p.seqY_id) y = &q;
                if (q.id == p.seqX_id) x = &q;
            }
            std::vector<int> ys, xs;
            if (substringWithHeader(y->seq, p.seqY_range, ys) != NwStat::success ||
                substringWithHeader(x->seq, p.seqX_range, xs) != NwStat::success)
                return (int)NwStat::errorInvalidValue;
            std::cout << "pair " << seqIdAndRangeToString(p.seqY_id, p.seqY_range) << " "
                      << seqIdAndRangeToString(p.seqX_id, p.seqX_range) << " " << ys.size() - 1 << " " << xs.size() - 1
                      << "\n";
        }
        return 0;
    }
    if (int st = gsa_ctx_create(a.device, &nw.ctx); st != GSA_SUCCESS)
    {
        std::cerr << "error: could not initialise HIP device " << a.device << "\n";
        return (int)NwStat::errorCudaGeneral;
    }
    nw.sm_count = gsa_device_cu_count(nw.ctx);

    std::ofstream resOfs, dbgOfs;
    if (open_out(a.resPath, resOfs) != NwStat::success)
    {
        std::cerr << "error: could not open resPath: \"" << a.resPath << "\"\n";
        gsa_ctx_destroy(nw.ctx);
        return (int)NwStat::errorIoStream;
    }
    if (!a.debugPath.empty() && open_out(a.debugPath, dbgOfs) != NwStat::success)
    {
        std::cerr << "error: could not open debugPath: \"" << a.debugPath << "\"\n";
        gsa_ctx_destroy(nw.ctx);
        return (int)NwStat::errorIoStream;
    }
    TsvPrintCtl ctl;
    ctl.fPrintScoreStats = a.fCalcScoreHash;
    ctl.fPrintTraceStats = a.fCalcTrace;
    {
        TsvPrintCtl hdr = ctl;
        hdr.writeColName = true;
        writeNwResultToTsv(resOfs, NwAlgResult {}, hdr);
    }
    ctl.writeValue = true;

    std::map<CompareKey, std::tuple<int, uint32_t, uint32_t>> compare;
    int calcErrors = 0;
    for (auto& algName : run)
    {
        if (a.fWriteProgress) std::cout << algName << ":\n" << std::flush;
        const NwAlgorithm& alg = algMap.at(algName);
        NwAlgParams params;
        for (auto& kv : paramData.paramMap)
            if (kv.first == algName) params = kv.second;
        for (auto& pair : pairs)
        {
            int iY = 0, iX = 0;
            for (size_t k = 0; k < seqs.size(); ++k)
            {
                if (seqs[k].id == pair.seqY_id) iY = (int)k;
                if (seqs[k].id == pair.seqX_id) iX = (int)k;
            }
            if (substringWithHeader(seqs[iY].seq, pair.seqY_range, nw.seqY) != NwStat::success ||
                substringWithHeader(seqs[iX].seq, pair.seqX_range, nw.seqX) != NwStat::success)
            {
                std::cerr << "error: cannot take substring of a sequence\n";
                gsa_ctx_destroy(nw.ctx);
                return (int)NwStat::errorInvalidValue;
            }
            nw.adjrows = (int)nw.seqY.size();
            nw.adjcols = (int)nw.seqX.size();
            for (params.reset(); params.hasCurr(); params.next())
            {
                std::vector<NwAlgResult> reps;
                for (int iR = -a.warmupPerAlign; iR < a.samplesPerAlign; ++iR)
                {
                    reps.emplace_back();
                    NwAlgResult& res = reps.back();
                    res.algName = algName;
                    res.algParams = params.copy();
                    res.algParamsJson = params.toJson();
                    res.seqY_idx = iY;
                    res.seqX_idx = iX;
                    res.seqY_id = seqs[iY].id;
                    res.seqX_id = seqs[iX].id;
                    res.seqY_range = pair.seqY_range;
                    res.seqX_range = pair.seqX_range;
                    res.seqY_len = nw.seqY.size() - 1;
                    res.seqX_len = nw.seqX.size() - 1;
                    res.substName = a.substName;
                    res.gapoCost = a.gapoCost;
                    res.warmup_runs = a.warmupPerAlign;
                    res.sample_runs = a.samplesPerAlign;
                    res.last_run_idx = iR;
                    res.sm_count = (size_t)nw.sm_count;

                    if ((res.stat = alg.align(params, nw, res)) != NwStat::success)
                        res.errstep = res.stat == NwStat::errorInvalidValue ? 1 : 2;
                    if (!res.errstep && a.fCalcScoreHash && (res.stat = alg.hash(nw, res)) != NwStat::success)
                        res.errstep = 3;
                    if (!res.errstep && a.fCalcTrace && (res.stat = alg.trace(nw, res, a.fPrintTrace)) != NwStat::success)
                        res.errstep = 4;
                    if (!res.errstep)
                    {
                        CompareKey key {res.seqY_id, res.seqX_id, pair.seqY_range.l, pair.seqY_range.r,
                                        pair.seqX_range.l, pair.seqX_range.r};
                        auto val = std::make_tuple(res.align_cost, res.score_hash, res.trace_hash);
                        auto it = compare.find(key);
                        if (it == compare.end())
                            compare[key] = val;
                        else if (it->second != val)
                        {
                            res.stat = NwStat::errorInvalidResult;
                            res.errstep = 5;
                            ++calcErrors;
                        }
                    }
                    if (!res.errstep && dbgOfs.is_open())
                    {
                        if (a.fPrintScore) alg.printScore(dbgOfs, nw, res);
                        if (a.fPrintTrace) alg.printTrace(dbgOfs, nw, res);
                    }
                    res.ramPeakAllocs = nw.measureHostAllocations();
                    if (iR < 0 && res.stat == NwStat::success) reps.pop_back();  // discard warmups
                    const bool last = iR == a.samplesPerAlign - 1 || res.stat != NwStat::success;
                    if (last && !reps.empty())
                    {
                        NwAlgResult out = reps.back();
                        std::vector<Laps> al, hs, tr;
                        for (auto& r : reps)
                        {
                            al.push_back(r.sw_align);
                            hs.push_back(r.sw_hash);
                            tr.push_back(r.sw_trace);
                        }
                        out.sw_align = Laps::combine(al);
                        out.sw_hash = Laps::combine(hs);
                        out.sw_trace = Laps::combine(tr);
                        writeNwResultToTsv(resOfs, out, ctl);
                        resOfs.flush();
                        if (a.fWriteProgress)
                            std::cout << "  " << seqIdAndRangeToString(out.seqY_id, out.seqY_range) << " x "
                                      << seqIdAndRangeToString(out.seqX_id, out.seqX_range) << " " << out.algParamsJson
                                      << ": " << (out.errstep ? nwStatName(out.stat) : "ok") << " cost "
                                      << out.align_cost << " calc " << out.sw_align.get_or_default("align.calc")
                                      << " ms\n"
                                      << std::flush;
                    }
                    nw.resetAllocsBenchmarkCycle();
                    if (res.stat != NwStat::success) break;
                }
            }
        }
    }
    gsa_ctx_destroy(nw.ctx);
    if (calcErrors)
    {
        std::cerr << "error: " << calcErrors << " result(s) differ from the reference algorithm\n";
        return (int)NwStat::errorInvalidResult;
    }
    return 0;
}
