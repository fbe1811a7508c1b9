// nw_host.cpp -- registry, align/trace/hash adapters over libgsa.so, input files and the
// TSV writer of the C++ host side (nw_host.hpp).
#include "nw_host.hpp"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <stdexcept>

#include "json_lite.hpp"

namespace gsa_host {

const char* nwStatName(NwStat s)
{
    static const char* names[] = {"success", "helpMenuRequested", "errorCudaGeneral", "errorMemoryAllocation",
                                  "errorMemoryTransfer", "errorKernelFailure", "errorIoStream", "errorInvalidFormat",
                                  "errorInvalidValue", "errorInvalidResult"};
    int i = (int)s;
    return (i >= 0 && i < 10) ? names[i] : "unknown";
}

// ---- NwAlgParams -------------------------------------------------------------------------
bool NwAlgParams::has(const std::string& name) const
{
    for (auto& p : params)
        if (p.first == name) return true;
    return false;
}

const NwAlgParam& NwAlgParams::at(const std::string& name) const
{
    for (auto& p : params)
        if (p.first == name) return p.second;
    throw std::out_of_range("no parameter " + name);
}

void NwAlgParams::next()
{
    // last parameter fastest; a wrapped parameter carries into the one before it
    for (auto it = params.rbegin(); it != params.rend(); ++it)
    {
        NwAlgParam& p = it->second;
        ++p.currIdx;
        if (p.hasCurr()) return;
        p.currIdx = 0;
    }
    isEnd = true;
}

void NwAlgParams::reset()
{
    for (auto& p : params) p.second.currIdx = 0;
    isEnd = false;
}

std::vector<std::pair<std::string, int>> NwAlgParams::copy() const
{
    std::vector<std::pair<std::string, int>> out;
    for (auto& p : params) out.emplace_back(p.first, p.second.curr());
    return out;
}

std::string NwAlgParams::toJson() const
{
    std::string s = "{";
    bool first = true;
    for (auto& p : params)
    {
        if (!first) s += ",";
        first = false;
        s += "\"" + p.first + "\":" + std::to_string(p.second.curr());
    }
    return s + "}";
}

// ---- Laps ----------------------------------------------------------------------------------
void Laps::add(const std::string& name, float ms)
{
    for (auto& l : laps)
        if (l.first == name)
        {
            l.second += ms;
            return;
        }
    laps.emplace_back(name, ms);
}

void Laps::lap(const std::string& name)
{
    const auto now = std::chrono::steady_clock::now();
    add(name, std::chrono::duration<float, std::milli>(now - mark).count());
    mark = now;
}

float Laps::get_or_default(const std::string& name) const
{
    for (auto& l : laps)
        if (l.first == name) return l.second;
    return 0.f;
}

Laps Laps::combine(const std::vector<Laps>& runs)
{
    Laps out;
    if (runs.empty()) return out;
    for (auto& r : runs)
        for (auto& l : r.laps) out.add(l.first, l.second);
    for (auto& l : out.laps) l.second /= (float)runs.size();
    return out;
}

// ---- NwAlgInput ----------------------------------------------------------------------------
size_t NwAlgInput::measureHostAllocations() const
{
    return (subst.capacity() + seqX.capacity() + seqY.capacity() + score.capacity() + tileHrowMat.capacity() +
            tileHcolMat.capacity()) *
           sizeof(int);
}

void NwAlgInput::resetAllocsBenchmarkCycle()
{
    score.clear();
    score.shrink_to_fit();
    tileHrowMat.clear();
    tileHrowMat.shrink_to_fit();
    tileHcolMat.clear();
    tileHcolMat.shrink_to_fit();
}

namespace {
using Clock = std::chrono::steady_clock;
float ms_since(Clock::time_point t0) { return std::chrono::duration<float, std::milli>(Clock::now() - t0).count(); }
}  // namespace

// The align adapters (NwAlign_Amd_Strip_*) are in nwalign_amd.cpp.

// ---- trace / hash adapters (the reference's L4 consumers, host C++ in libgsa) -------------
NwStat NwHash1_Plain(NwAlgInput& nw, NwAlgResult& res)
{
    if (nw.score.size() != (size_t)nw.adjrows * (size_t)nw.adjcols) return NwStat::errorInvalidValue;
    auto t0 = Clock::now();
    res.score_hash = gsa_hash_full(nw.score.data(), nw.adjrows, nw.adjcols);
    res.sw_hash.add("hash.calc", ms_since(t0));
    return NwStat::success;
}

NwStat NwTrace1_Plain(NwAlgInput& nw, NwAlgResult& res, bool)
{
    if (nw.score.size() != (size_t)nw.adjrows * (size_t)nw.adjcols) return NwStat::errorInvalidValue;
    auto t0 = Clock::now();
    const int64_t cap = 16 * ((int64_t)nw.adjrows + nw.adjcols) + 64;
    std::string edit((size_t)cap, '\0');
    res.sw_trace.add("trace.alloc", ms_since(t0));
    t0 = Clock::now();
    int64_t len = 0;
    uint32_t th = 0;
    int st = gsa_trace_full(nw.score.data(), nw.seqY.data(), nw.adjrows, nw.seqX.data(), nw.adjcols, &edit[0], cap, &len,
                            &th);
    res.sw_trace.add("trace.calc", ms_since(t0));
    if (st != GSA_SUCCESS) return (NwStat)st;
    edit.resize((size_t)len);
    res.edit_trace = std::move(edit);
    res.trace_hash = th;
    return NwStat::success;
}

NwStat NwHash2_Sparse(NwAlgInput& nw, NwAlgResult& res)
{
    if (nw.tileHrowMat.empty()) return NwStat::errorInvalidValue;
    auto t0 = Clock::now();
    res.score_hash = gsa_hash_sparse(nw.tileHrowMat.data(), nw.tileHcolMat.data(), &nw.geom, nw.seqY.data(), nw.adjrows,
                                     nw.seqX.data(), nw.adjcols, nw.subst.data(), nw.substsz, nw.gapoCost);
    res.sw_hash.add("hash.calc", ms_since(t0));
    return NwStat::success;
}

NwStat NwTrace2_Sparse(NwAlgInput& nw, NwAlgResult& res, bool)
{
    if (nw.tileHrowMat.empty()) return NwStat::errorInvalidValue;
    auto t0 = Clock::now();
    const int64_t cap = 16 * ((int64_t)nw.adjrows + nw.adjcols) + 64;
    std::string edit((size_t)cap, '\0');
    res.sw_trace.add("trace.alloc", ms_since(t0));
    t0 = Clock::now();
    int64_t len = 0;
    uint32_t th = 0;
    int32_t cost = 0;
    int st = gsa_trace_sparse(nw.tileHrowMat.data(), nw.tileHcolMat.data(), &nw.geom, nw.seqY.data(), nw.adjrows,
                              nw.seqX.data(), nw.adjcols, nw.subst.data(), nw.substsz, nw.gapoCost, &edit[0], cap, &len,
                              &th, &cost);
    res.sw_trace.add("trace.calc", ms_since(t0));
    if (st != GSA_SUCCESS) return (NwStat)st;
    edit.resize((size_t)len);
    res.edit_trace = std::move(edit);
    res.trace_hash = th;
    return NwStat::success;
}

NwStat NwPrintScore1_Plain(std::ostream& os, const NwAlgInput& nw, NwAlgResult&)
{
    if (nw.score.size() != (size_t)nw.adjrows * (size_t)nw.adjcols) return NwStat::errorInvalidValue;
    for (int i = 0; i < nw.adjrows; ++i)
    {
        for (int j = 0; j < nw.adjcols; ++j) os << std::setw(5) << nw.score[(size_t)i * nw.adjcols + j] << (j + 1 < nw.adjcols ? "," : "");
        os << '\n';
    }
    return os ? NwStat::success : NwStat::errorIoStream;
}

NwStat NwPrintScore2_Sparse(std::ostream& os, const NwAlgInput& nw, NwAlgResult&)
{
    // tile header rows then columns, one tile per line
    const auto& g = nw.geom;
    for (int64_t k = 0; k < (int64_t)g.tileHdrMatRows * g.tileHdrMatCols; ++k)
    {
        os << "tile " << k / g.tileHdrMatCols << "," << k % g.tileHdrMatCols << " hrow:";
        for (int e = 0; e < g.tileHrowLen; ++e) os << ' ' << nw.tileHrowMat[(size_t)k * g.tileHrowLen + e];
        os << " | hcol:";
        for (int e = 0; e < g.tileHcolLen; ++e) os << ' ' << nw.tileHcolMat[(size_t)k * g.tileHcolLen + e];
        os << '\n';
    }
    return os ? NwStat::success : NwStat::errorIoStream;
}

NwStat NwPrintTrace1_Plain(std::ostream& os, const NwAlgInput&, const NwAlgResult& res)
{
    os << res.edit_trace << '\n';
    return os ? NwStat::success : NwStat::errorIoStream;
}

void getNwAlgorithmMap(std::map<std::string, NwAlgorithm>& algMap)
{
    auto plain = [](NwAlgorithm::NwAlignFn f) {
        return NwAlgorithm {f, NwTrace1_Plain, NwHash1_Plain, NwPrintScore1_Plain, NwPrintTrace1_Plain};
    };
    auto sparse = [](NwAlgorithm::NwAlignFn f) {
        return NwAlgorithm {f, NwTrace2_Sparse, NwHash2_Sparse, NwPrintScore2_Sparse, NwPrintTrace1_Plain};
    };
    std::map<std::string, NwAlgorithm> m {
        {"NwAlign_Gpu1_Ml_Diag", plain(NwAlign_Gpu1_Ml_Diag)},
        {"NwAlign_Gpu2_Ml_DiagRow2Pass", plain(NwAlign_Gpu2_Ml_DiagRow2Pass)},
        {"NwAlign_Gpu3_Ml_DiagDiag", plain(NwAlign_Gpu3_Ml_DiagDiag)},
        {"NwAlign_Gpu4_Ml_DiagDiag2Pass", plain(NwAlign_Gpu4_Ml_DiagDiag2Pass)},
        {"NwAlign_Gpu5_Coop_DiagDiag", plain(NwAlign_Gpu5_Coop_DiagDiag)},
        {"NwAlign_Gpu6_Coop_DiagDiag2Pass", plain(NwAlign_Gpu6_Coop_DiagDiag2Pass)},
        {"NwAlign_Gpu7_Mlsp_DiagDiag", sparse(NwAlign_Gpu7_Mlsp_DiagDiag)},
        {"NwAlign_Gpu8_Mlsp_DiagDiag", sparse(NwAlign_Gpu8_Mlsp_DiagDiag)},
        {"NwAlign_Gpu9_Mlsp_DiagDiagDiag", sparse(NwAlign_Gpu9_Mlsp_DiagDiagDiag)},
        {"NwAlign_Amd_Strip_Full", plain(NwAlign_Amd_Strip_Full)},
        {"NwAlign_Amd_Strip_Mlsp", sparse(NwAlign_Amd_Strip_Mlsp)},
        {"NwAlign_Amd_Strip_Mlsppt", sparse(NwAlign_Amd_Strip_Mlsppt)},
    };
    algMap.swap(m);
}

// ---- input files ---------------------------------------------------------------------------
namespace {

NwStat read_text(const std::string& path, std::string& text, std::string& err)
{
    std::ifstream f(path, std::ios::binary);
    if (!f)
    {
        err = path + ": could not open file";
        return NwStat::errorIoStream;
    }
    std::ostringstream ss;
    ss << f.rdbuf();
    text = ss.str();
    return NwStat::success;
}

}  // namespace

int NwSubstData::letterIndex(char c) const
{
    for (auto& kv : letterMap)
        if (kv.first == c) return kv.second;
    return -1;
}

NwStat readSubstFile(const std::string& path, NwSubstData& out, std::string& err)
{
    std::string text;
    if (NwStat s = read_text(path, text, err); s != NwStat::success) return s;
    Json j;
    try
    {
        j = parse_json(text);
    }
    catch (const JsonError& e)
    {
        err = path + ":" + e.what();
        return NwStat::errorInvalidFormat;
    }
    const Json* lm = j.find("letterMap");
    const Json* sm = j.find("substMap");
    if (!j.is_object() || !lm || !lm->is_object() || !sm || !sm->is_object())
    {
        err = path + ": expected object with \"letterMap\" and \"substMap\"";
        return NwStat::errorInvalidFormat;
    }
    NwSubstData d;
    int idx = 0;
    for (auto& kv : lm->obj)
    {
        if (kv.first.size() != 1 || !kv.second.is_int())
        {
            err = path + ": letter map entries must be single characters mapped to integers";
            return NwStat::errorInvalidFormat;
        }
        if (kv.second.i != idx)  // src/cmd_parser.cpp:316-335
        {
            err = path + ": letter map values must be consecutive starting from 0";
            return NwStat::errorInvalidFormat;
        }
        d.letterMap.emplace_back(kv.first[0], idx++);
    }
    const size_t n = d.letterMap.size();
    for (auto& kv : sm->obj)
    {
        std::vector<int> v;
        if (kv.second.is_array())
            for (auto& e : kv.second.arr)
            {
                if (!e.is_int())
                {
                    err = path + ": substitution matrix \"" + kv.first + "\" must hold integers";
                    return NwStat::errorInvalidFormat;
                }
                v.push_back((int)e.i);
            }
        if (v.size() != n * n)  // src/cmd_parser.cpp:337-355
        {
            err = path + ": substitution matrix \"" + kv.first + "\" must have " + std::to_string(n) + "x" +
                  std::to_string(n) + " elements";
            return NwStat::errorInvalidFormat;
        }
        d.substMap.emplace_back(kv.first, std::move(v));
    }
    out = std::move(d);
    return NwStat::success;
}

NwStat readAlgParamsFile(const std::string& path, NwAlgParamsData& out, std::string& err)
{
    std::string text;
    if (NwStat s = read_text(path, text, err); s != NwStat::success) return s;
    Json j;
    try
    {
        j = parse_json(text);
    }
    catch (const JsonError& e)
    {
        err = path + ":" + e.what();
        return NwStat::errorInvalidFormat;
    }
    if (!j.is_object())
    {
        err = path + ": expected an object of algorithm names";
        return NwStat::errorInvalidFormat;
    }
    NwAlgParamsData d;
    for (auto& alg : j.obj)
    {
        if (!alg.second.is_object())
        {
            err = path + ": parameters of \"" + alg.first + "\" must be an object";
            return NwStat::errorInvalidFormat;
        }
        NwAlgParams p;
        for (auto& prm : alg.second.obj)
        {
            NwAlgParam one;
            if (!prm.second.is_array() || prm.second.arr.empty())
            {
                err = path + ": parameter \"" + prm.first + "\" of \"" + alg.first + "\" must be a non-empty array";
                return NwStat::errorInvalidFormat;
            }
            for (auto& v : prm.second.arr)
            {
                if (!v.is_int())
                {
                    err = path + ": parameter values must be integers";
                    return NwStat::errorInvalidFormat;
                }
                one.values.push_back((int)v.i);
            }
            p.params.emplace_back(prm.first, std::move(one));
        }
        d.paramMap.emplace_back(alg.first, std::move(p));
    }
    out = std::move(d);
    return NwStat::success;
}

NwStat readFastaFile(const std::string& path, const NwSubstData& subst, std::vector<NwSeq>& out, std::string& err)
{
    std::ifstream f(path);
    if (!f)
    {
        err = path + ": could not open file";
        return NwStat::errorIoStream;
    }
    std::vector<NwSeq> seqs;
    std::string line;
    int iline = 0;
    enum { kHeader, kSequence, kSeqOrHeader } state = kHeader;
    auto fmt = [&](int col, const std::string& m) {
        err = path + ":" + std::to_string(iline) + ":" + std::to_string(col) + ": " + m;
        return NwStat::errorInvalidFormat;
    };
    while (std::getline(f, line))
    {
        ++iline;
        size_t a = line.find_first_not_of(" \t\r");
        if (a == std::string::npos) continue;
        if (line[a] == '>')
        {
            if (state == kSequence) return fmt((int)a + 1, "expected sequence after header");
            std::istringstream hs(line.substr(a + 1));
            NwSeq s;
            if (!(hs >> s.id)) return fmt((int)a + 2, "expected sequence id after '>' symbol");
            for (auto& q : seqs)
                if (q.id == s.id) return fmt((int)a + 2, "duplicate sequence id");
            std::getline(hs >> std::ws, s.info);
            while (!s.info.empty() && std::isspace((unsigned char)s.info.back())) s.info.pop_back();
            s.seq.push_back(0);  // header element (src/file_formats.cpp:43-47)
            seqs.push_back(std::move(s));
            state = kSequence;
            continue;
        }
        if (state == kHeader) return fmt((int)a + 1, "expected sequence header (>)");
        for (size_t c = 0; c < line.size(); ++c)
        {
            char ch = line[c];
            if (std::isspace((unsigned char)ch)) continue;
            int v = subst.letterIndex(ch);
            if (v < 0) return fmt((int)c + 1, "letter not found in substitution letters");
            seqs.back().seq.push_back(v);
        }
        state = kSeqOrHeader;
    }
    if (state == kSequence)
    {
        err = path + ": expected sequence after header";
        return NwStat::errorInvalidFormat;
    }
    if (state == kHeader)
    {
        err = path + ": expected sequence header (>)";
        return NwStat::errorInvalidFormat;
    }
    out = std::move(seqs);
    return NwStat::success;
}

namespace {

// "id" or "id[l:r]" with either bound optional, at line[pos...]; advances pos
NwStat parse_id_range(const std::string& line, size_t& pos, const std::vector<NwSeq>& seqs, std::string& id,
                      NwRange& rng, std::string& msg)
{
    while (pos < line.size() && std::isspace((unsigned char)line[pos])) ++pos;
    size_t b = pos;
    while (pos < line.size() && !std::isspace((unsigned char)line[pos]) && line[pos] != '[') ++pos;
    if (pos == b)
    {
        msg = "expected sequence id";
        return NwStat::errorInvalidFormat;
    }
    id = line.substr(b, pos - b);
    const NwSeq* s = nullptr;
    for (auto& q : seqs)
        if (q.id == id) s = &q;
    if (!s)
    {
        msg = "unknown sequence id";
        return NwStat::errorInvalidFormat;
    }
    const int64_t n = (int64_t)s->seq.size() - 1;
    rng = NwRange {false, false, 0, n};
    if (pos < line.size() && line[pos] == '[')
    {
        size_t e = line.find(']', pos);
        size_t c = line.find(':', pos);
        if (e == std::string::npos || c == std::string::npos || c > e)
        {
            msg = "expected [l:r] range";
            return NwStat::errorInvalidFormat;
        }
        auto num = [&](size_t x, size_t y, int64_t& v) {
            std::string t = line.substr(x, y - x);
            size_t a = t.find_first_not_of(" \t"), z = t.find_last_not_of(" \t");
            if (a == std::string::npos) return false;
            v = std::stoll(t.substr(a, z - a + 1));
            return true;
        };
        try
        {
            if (num(pos + 1, c, rng.l)) rng.lNotDefault = true;
            if (num(c + 1, e, rng.r)) rng.rNotDefault = true;
        }
        catch (const std::exception&)
        {
            msg = "expected integer range bounds";
            return NwStat::errorInvalidFormat;
        }
        if (rng.l < 0 || rng.l >= n)
        {
            msg = "left bound out of range";
            return NwStat::errorInvalidFormat;
        }
        if (rng.r <= rng.l || rng.r > n)
        {
            msg = "right bound out of range";
            return NwStat::errorInvalidFormat;
        }
        pos = e + 1;
    }
    return NwStat::success;
}

}  // namespace

NwStat readSeqPairFile(const std::string& path, const std::vector<NwSeq>& seqs, std::vector<NwSeqPair>& out,
                       std::string& err)
{
    std::ifstream f(path);
    if (!f)
    {
        err = path + ": could not open file";
        return NwStat::errorIoStream;
    }
    std::vector<NwSeqPair> pairs;
    std::string line;
    int iline = 0;
    while (std::getline(f, line))
    {
        ++iline;
        if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
        NwSeqPair p;
        size_t pos = 0;
        std::string msg;
        if (parse_id_range(line, pos, seqs, p.seqY_id, p.seqY_range, msg) != NwStat::success ||
            parse_id_range(line, pos, seqs, p.seqX_id, p.seqX_range, msg) != NwStat::success)
        {
            err = path + ":" + std::to_string(iline) + ":" + std::to_string(pos + 1) + ": " + msg;
            return NwStat::errorInvalidFormat;
        }
        if (line.find_first_not_of(" \t\r", pos) != std::string::npos)
        {
            err = path + ":" + std::to_string(iline) + ":" + std::to_string(pos + 1) + ": expected next line";
            return NwStat::errorInvalidFormat;
        }
        pairs.push_back(std::move(p));
    }
    if (pairs.empty())
    {
        err = path + ": expected at least one sequence pair";
        return NwStat::errorInvalidFormat;
    }
    out = std::move(pairs);
    return NwStat::success;
}

NwStat substringWithHeader(const std::vector<int>& seq, const NwRange& r, std::vector<int>& out)
{
    const int64_t n = (int64_t)seq.size() - 1;
    if (r.l < 0 || r.l >= n || r.r <= r.l || r.r > n) return NwStat::errorInvalidValue;
    out.assign(1, 0);
    out.insert(out.end(), seq.begin() + 1 + r.l, seq.begin() + 1 + r.r);
    return NwStat::success;
}

std::string seqIdAndRangeToString(const std::string& id, const NwRange& r)
{
    if (!r.lNotDefault && !r.rNotDefault) return id;
    std::string s = id + "[";
    if (r.lNotDefault) s += std::to_string(r.l);
    s += ":";
    if (r.rNotDefault) s += std::to_string(r.r);
    return s + "]";
}

// ---- TSV -------------------------------------------------------------------------------------
NwStat writeNwResultToTsv(std::ostream& os, const NwAlgResult& res, const TsvPrintCtl& ctl)
{
    if (ctl.writeColName == ctl.writeValue) return NwStat::errorInvalidValue;
    bool first = true;
    auto field = [&](const char* name, auto value) {
        if (!first) os << '\t';
        first = false;
        if (ctl.writeColName)
            os << name;
        else
            os << value;
    };
    auto hex = [](uint32_t v) {
        std::ostringstream s;
        s << std::hex << std::setw(8) << std::setfill('0') << v;
        return s.str();
    };
    auto ms = [](float v) {
        std::ostringstream s;
        s << std::fixed << std::setprecision(4) << v;
        return s.str();
    };
    field("alg_name", res.algName);
    field("seqY_idx", res.seqY_idx);
    field("seqX_idx", res.seqX_idx);
    field("seqY_id", seqIdAndRangeToString(res.seqY_id, res.seqY_range));
    field("seqX_id", seqIdAndRangeToString(res.seqX_id, res.seqX_range));
    field("seqY_len", res.seqY_len);
    field("seqX_len", res.seqX_len);
    field("subst_name", res.substName);
    field("gapo_cost", res.gapoCost);
    field("warmup_runs", res.warmup_runs);
    field("sample_runs", res.sample_runs);
    field("last_run_idx", res.last_run_idx);
    field("alg_params", res.algParamsJson);
    field("err_step", res.errstep);
    field("nw_stat", (int)res.stat);
    field("cuda_stat", res.hipStat);
    field("align_cost", res.align_cost);
    if (ctl.fPrintScoreStats) field("score_hash", hex(res.score_hash));
    if (ctl.fPrintTraceStats) field("trace_hash", hex(res.trace_hash));
    field("sm_count", res.sm_count);
    field("ram_peak_allocs", res.ramPeakAllocs);
    field("glmem_peak_allocs", res.globalMemPeakAllocs);
    field("shmem_peak_allocs", res.sharedMemPeakAllocs);
    field("locmem_peak_allocs", res.localMemPeakAllocs);
    field("regmem_peak_allocs", res.regMemPeakAllocs);
    field("align.alloc", ms(res.sw_align.get_or_default("align.alloc")));
    field("align.cpy_dev", ms(res.sw_align.get_or_default("align.cpy_dev")));
    field("align.init_hdr", ms(res.sw_align.get_or_default("align.init_hdr")));
    field("align.calc_init", ms(res.sw_align.get_or_default("align.calc_init")));
    field("align.calc", ms(res.sw_align.get_or_default("align.calc")));
    field("align.cpy_host", ms(res.sw_align.get_or_default("align.cpy_host")));
    if (ctl.fPrintScoreStats) field("hash.calc", ms(res.sw_hash.get_or_default("hash.calc")));
    if (ctl.fPrintTraceStats)
    {
        field("trace.alloc", ms(res.sw_trace.get_or_default("trace.alloc")));
        field("trace.calc", ms(res.sw_trace.get_or_default("trace.calc")));
        field("edit_trace", res.edit_trace);
    }
    os << '\n';
    return os ? NwStat::success : NwStat::errorIoStream;
}

}  // namespace gsa_host
