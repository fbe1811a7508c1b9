// nw_host.hpp -- C++ host side of the MI355X engine, mirroring the reference's align-path
// interface so a GpuSeqAlign user finds the same objects, names and error behaviour:
//   NwStat                      src/run_types.hpp:12-24
//   NwRange / NwAlgParam(s)      src/run_types.hpp:26-66
//   NwAlgInput / NwAlgResult     src/run_types.hpp:68-150
//   NwAlgorithm + registry       src/nw_algorithm.hpp:8-44, src/nw_algorithm.cpp:48-69
//   input files / TSV results    src/file_formats.cpp:143-524, src/cmd_parser.cpp:316-355
// Everything on the device goes through the C ABI of libgsa.so (include/gsa.h); this layer
// holds host buffers, parameters, timings and the benchmark bookkeeping only.
#pragma once

#include <chrono>
#include <cstdint>
#include <map>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gsa.h"

namespace gsa_host {

enum class NwStat : int
{
    success,
    helpMenuRequested,
    errorCudaGeneral,  // HIP runtime failure (name kept for drop-in compatibility)
    errorMemoryAllocation,
    errorMemoryTransfer,
    errorKernelFailure,
    errorIoStream,
    errorInvalidFormat,
    errorInvalidValue,
    errorInvalidResult,
};
static_assert((int)NwStat::errorInvalidResult == GSA_ERROR_INVALID_RESULT, "NwStat mirrors gsa_stat");

const char* nwStatName(NwStat s);

// Sequence substring [l, r), with "given explicitly" flags (src/run_types.hpp:26-35).
struct NwRange
{
    bool lNotDefault = false;
    bool rNotDefault = false;
    int64_t l = 0;
    int64_t r = 0;
    bool operator==(const NwRange& o) const
    {
        return lNotDefault == o.lNotDefault && rNotDefault == o.rNotDefault && l == o.l && r == o.r;
    }
};

// One parameter with its candidate values (src/run_types.hpp:37-50).
struct NwAlgParam
{
    std::vector<int> values;
    size_t currIdx = 0;
    int curr() const { return values.at(currIdx); }
    bool hasCurr() const { return currIdx < values.size(); }
};

// Named parameters iterated as a Cartesian product, last parameter fastest
// (src/run_types.hpp:52-66; src/run_types.cpp NwAlgParams::next).
struct NwAlgParams
{
    std::vector<std::pair<std::string, NwAlgParam>> params;  // file order
    bool isEnd = false;

    bool has(const std::string& name) const;
    const NwAlgParam& at(const std::string& name) const;  // throws std::out_of_range
    bool hasCurr() const { return !isEnd; }
    void next();
    void reset();
    std::vector<std::pair<std::string, int>> copy() const;
    std::string toJson() const;  // {"name":value,...} as the TSV alg_params column
};

// Stopwatch laps in ms, accumulated per name (src/stopwatch.hpp:10-33, stopwatch.cpp:4-50):
// start() sets the mark, lap(name) adds the time since the mark to `name` and moves the mark.
struct Laps
{
    std::vector<std::pair<std::string, float>> laps;
    std::chrono::steady_clock::time_point mark {};
    void start() { mark = std::chrono::steady_clock::now(); }
    void lap(const std::string& name);
    void add(const std::string& name, float ms);
    float get_or_default(const std::string& name) const;
    static Laps combine(const std::vector<Laps>& runs);  // per-name average
};
using Stopwatch = Laps;  // the reference's name

struct NwAlgInput
{
    std::vector<int> subst;
    std::vector<int> seqX;  // element 0 = header (src/file_formats.cpp:43-47)
    std::vector<int> seqY;
    std::vector<int> score;        // plain family: adjrows*adjcols
    std::vector<int> tileHrowMat;  // sparse family
    std::vector<int> tileHcolMat;
    gsa_sparse_geom geom {};

    int substsz = 0;
    int adjrows = 0;
    int adjcols = 0;
    int gapoCost = -11;
    int tileHdrMatRows = 0;
    int tileHdrMatCols = 0;
    int tileHrowLen = 0;
    int tileHcolLen = 0;

    int sm_count = 0;  // CU count of the device
    gsa_ctx* ctx = nullptr;  // device context (the reference keeps device buffers here)

    size_t measureHostAllocations() const;
    void resetAllocsBenchmarkCycle();  // src/run_types.cpp:143-168
};

struct NwAlgResult
{
    std::string algName;
    std::vector<std::pair<std::string, int>> algParams;
    std::string algParamsJson = "{}";
    int seqY_idx = 0;
    int seqX_idx = 0;
    std::string seqY_id;
    std::string seqX_id;
    NwRange seqY_range;
    NwRange seqX_range;

    int errstep = 0;  // 0 for success
    NwStat stat = NwStat::success;
    int hipStat = 0;  // raw hipError_t of the failing runtime call (reference: cudaStat)

    size_t seqY_len = 0;
    size_t seqX_len = 0;
    std::string substName;
    int gapoCost = 0;
    int warmup_runs = 0;
    int sample_runs = 0;
    int last_run_idx = 0;

    int align_cost = 0;
    uint32_t score_hash = 0;
    uint32_t trace_hash = 0;
    std::string edit_trace;

    size_t sm_count = 0;
    size_t ramPeakAllocs = 0;
    size_t globalMemPeakAllocs = 0;
    size_t sharedMemPeakAllocs = 0;
    size_t localMemPeakAllocs = 0;
    size_t regMemPeakAllocs = 0;

    Laps sw_align, sw_hash, sw_trace;
};

// {align, trace, hash, printScore, printTrace} of one algorithm (src/nw_algorithm.hpp:8-44).
class NwAlgorithm
{
public:
    using NwAlignFn = NwStat (*)(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
    using NwTraceFn = NwStat (*)(NwAlgInput& nw, NwAlgResult& res, bool calcDebugTrace);
    using NwHashFn = NwStat (*)(NwAlgInput& nw, NwAlgResult& res);
    using NwPrintScoreFn = NwStat (*)(std::ostream& os, const NwAlgInput& nw, NwAlgResult& res);
    using NwPrintTraceFn = NwStat (*)(std::ostream& os, const NwAlgInput& nw, const NwAlgResult& res);

    NwAlgorithm() = default;
    NwAlgorithm(NwAlignFn a, NwTraceFn t, NwHashFn h, NwPrintScoreFn ps, NwPrintTraceFn pt)
        : align_(a), trace_(t), hash_(h), printScore_(ps), printTrace_(pt)
    {
    }
    NwStat align(const NwAlgParams& p, NwAlgInput& nw, NwAlgResult& res) const { return align_(p, nw, res); }
    NwStat trace(NwAlgInput& nw, NwAlgResult& res, bool dbg) const { return trace_(nw, res, dbg); }
    NwStat hash(NwAlgInput& nw, NwAlgResult& res) const { return hash_(nw, res); }
    NwStat printScore(std::ostream& os, const NwAlgInput& nw, NwAlgResult& res) const
    {
        return printScore_(os, nw, res);
    }
    NwStat printTrace(std::ostream& os, const NwAlgInput& nw, const NwAlgResult& res) const
    {
        return printTrace_(os, nw, res);
    }

private:
    NwAlignFn align_ = nullptr;
    NwTraceFn trace_ = nullptr;
    NwHashFn hash_ = nullptr;
    NwPrintScoreFn printScore_ = nullptr;
    NwPrintTraceFn printTrace_ = nullptr;
};

// The reference's algorithm names that this engine serves (plain family NwAlign_Gpu1..6,
// sparse family NwAlign_Gpu7..9) plus this engine's own names.  The CPU algorithms
// NwAlign_Cpu1..4 are the reference's oracle and baseline, not part of the GPU path: they
// are absent here ("out of scope").
void getNwAlgorithmMap(std::map<std::string, NwAlgorithm>& algMap);

// Individual functions (the reference's nw_fns.hpp names): one align adapter per slot name, each
// with the parameter rules of the reference's function of that name (nwalign_amd.cpp).
NwStat NwAlign_Gpu1_Ml_Diag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu2_Ml_DiagRow2Pass(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu3_Ml_DiagDiag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu4_Ml_DiagDiag2Pass(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu5_Coop_DiagDiag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu6_Coop_DiagDiag2Pass(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu7_Mlsp_DiagDiag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu8_Mlsp_DiagDiag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Gpu9_Mlsp_DiagDiagDiag(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Amd_Strip_Full(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Amd_Strip_Mlsp(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
NwStat NwAlign_Amd_Strip_Mlsppt(const NwAlgParams& pr, NwAlgInput& nw, NwAlgResult& res);
// The engine geometry a slot's parameters select (no device needed): errorInvalidValue where
// the reference's function of that name rejects them; sparse slots give the tile width.
struct SlotGeometry
{
    bool sparse = false;
    int tileBx = 0;  // sparse: the engine's tile width (tile height: gsa_sparse_tile_by())
};
NwStat slotGeometry(const std::string& slot, const NwAlgParams& pr, SlotGeometry& out);
NwStat NwTrace1_Plain(NwAlgInput& nw, NwAlgResult& res, bool calcDebugTrace);
NwStat NwHash1_Plain(NwAlgInput& nw, NwAlgResult& res);
NwStat NwTrace2_Sparse(NwAlgInput& nw, NwAlgResult& res, bool calcDebugTrace);
NwStat NwHash2_Sparse(NwAlgInput& nw, NwAlgResult& res);
NwStat NwPrintScore1_Plain(std::ostream& os, const NwAlgInput& nw, NwAlgResult& res);
NwStat NwPrintScore2_Sparse(std::ostream& os, const NwAlgInput& nw, NwAlgResult& res);
NwStat NwPrintTrace1_Plain(std::ostream& os, const NwAlgInput& nw, const NwAlgResult& res);

// ---- input files (src/file_formats.cpp, src/cmd_parser.cpp:316-355) ---------------------
struct NwSubstData
{
    std::vector<std::pair<char, int>> letterMap;
    std::vector<std::pair<std::string, std::vector<int>>> substMap;
    int letterIndex(char c) const;  // -1 if absent
};
struct NwAlgParamsData
{
    std::vector<std::pair<std::string, NwAlgParams>> paramMap;  // file order
};
struct NwSeq
{
    std::string id;
    std::string info;
    std::vector<int> seq;  // element 0 = header
};
struct NwSeqPair
{
    std::string seqY_id;
    std::string seqX_id;
    NwRange seqY_range;
    NwRange seqX_range;
};

// Each reader returns success or errorIoStream / errorInvalidFormat with a message in `err`
// shaped "path:line:col: message" like the reference (src/file_formats.cpp:15-31).
NwStat readSubstFile(const std::string& path, NwSubstData& out, std::string& err);
NwStat readAlgParamsFile(const std::string& path, NwAlgParamsData& out, std::string& err);
NwStat readFastaFile(const std::string& path, const NwSubstData& subst, std::vector<NwSeq>& out, std::string& err);
NwStat readSeqPairFile(const std::string& path, const std::vector<NwSeq>& seqs, std::vector<NwSeqPair>& out,
                       std::string& err);
// vectorSubstringWithHeader (src/benchmark.cpp:14-36)
NwStat substringWithHeader(const std::vector<int>& seq, const NwRange& r, std::vector<int>& out);
std::string seqIdAndRangeToString(const std::string& id, const NwRange& r);

struct TsvPrintCtl
{
    bool writeColName = false;
    bool writeValue = false;
    bool fPrintScoreStats = false;
    bool fPrintTraceStats = false;
};
// writeNwResultToTsv (src/file_formats.cpp:455-524): same columns, same formatting.
NwStat writeNwResultToTsv(std::ostream& os, const NwAlgResult& res, const TsvPrintCtl& ctl);

}  // namespace gsa_host
