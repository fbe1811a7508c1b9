"""C++ host side (gpuseqalign_amd/host): the `gsa_nw` bench driver with the reference's CLI,
input readers, parameter iteration and TSV writer (nw_host.hpp).

CPU tests use --dryRun (every input read and checked, no device touched); the GPU test runs
the reference's own pair files end to end and checks the TSV against the reference's known
answers, with the plain and the sparse family verifying each other exactly as
the reference driver's setOrVerifyResult does (src/benchmark.cpp:120-147).
"""
import csv
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RES = os.path.join(ROOT, "tests", "golden", "resrc")
BIN = os.path.join(ROOT, "gpuseqalign_amd", "bin", "gsa_nw")


@pytest.fixture(scope="module")
def gsa_nw():
    if not os.path.exists(os.path.join(ROOT, "gpuseqalign_amd", "libgsa.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "gpuseqalign_amd", "csrc")])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "gpuseqalign_amd", "host")])
    return BIN


def run(binary, *args, cwd=None):
    return subprocess.run([binary, *args], capture_output=True, text=True, cwd=cwd, timeout=600)


def base_args():
    return ["-b", os.path.join(RES, "subst.json"), "-r", os.path.join(RES, "param_best.json"),
            "-s", os.path.join(RES, "seq_generated.fa")]


def test_help_and_missing_args(gsa_nw):
    r = run(gsa_nw, "--help")
    assert r.returncode == 0 and "--algParamPath" in r.stdout
    r = run(gsa_nw)
    assert r.returncode == 8  # errorInvalidValue, as the reference driver
    r = run(gsa_nw, "-r", "x.json")
    assert r.returncode == 8 and "--seqPath" in r.stderr
    r = run(gsa_nw, "--bogus")
    assert r.returncode == 8 and "unknown parameter" in r.stderr


def test_dry_run_reads_reference_inputs(gsa_nw):
    r = run(gsa_nw, *base_args(), "-p", os.path.join(RES, "pair_debug.txt"), "--dryRun")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    pairs = [l for l in lines if l.startswith("pair ")]
    with open(os.path.join(RES, "pair_debug.txt")) as f:
        n_expected = sum(1 for l in f if l.strip())
    assert len(pairs) == n_expected
    algs = [l.split()[1] for l in lines if l.startswith("alg ")]
    # the reference's GPU names are served; its CPU oracle family is skipped with a warning
    assert "NwAlign_Gpu3_Ml_DiagDiag" in algs and "NwAlign_Gpu9_Mlsp_DiagDiagDiag" in algs
    assert not any(a.startswith("NwAlign_Cpu") for a in algs)
    assert "NwAlign_Cpu1_St_Row" in r.stderr


def test_dry_run_ranges_and_default_pairs(gsa_nw, tmp_path):
    pf = tmp_path / "p.txt"
    pf.write_text("len12124[:10000] len15390[:10000]\nlen31[1:] len32[:5]\n")
    r = run(gsa_nw, *base_args(), "-p", str(pf), "--dryRun", "--algName", "NwAlign_Gpu3_Ml_DiagDiag")
    assert r.returncode == 0, r.stderr
    pairs = [l.split() for l in r.stdout.splitlines() if l.startswith("pair ")]
    assert pairs == [["pair", "len12124[:10000]", "len15390[:10000]", "10000", "10000"],
                     ["pair", "len31[1:]", "len32[:5]", "30", "5"]]
    # no pair file: every sequence against the first one
    r = run(gsa_nw, *base_args(), "--dryRun", "--algName", "NwAlign_Gpu3_Ml_DiagDiag")
    assert r.returncode == 0
    assert len([l for l in r.stdout.splitlines() if l.startswith("pair ")]) > 1


def test_param_combinations(gsa_nw, tmp_path):
    pj = tmp_path / "params.json"
    pj.write_text('// comment allowed\n{"NwAlign_Amd_Strip_Mlsp": {"tileBx": [64, 128, 256], "x": [1, 2]},\n'
                  ' "NwAlign_Gpu3_Ml_DiagDiag": {"threadsPerBlockA": [96], "tileBx": [54]}}')
    r = run(gsa_nw, "-b", os.path.join(RES, "subst.json"), "-r", str(pj), "-s", os.path.join(RES, "seq_generated.fa"),
            "--dryRun")
    assert r.returncode == 0, r.stderr
    combos = {l.split()[1]: int(l.split()[3]) for l in r.stdout.splitlines() if l.startswith("alg ")}
    assert combos == {"NwAlign_Amd_Strip_Mlsp": 6, "NwAlign_Gpu3_Ml_DiagDiag": 1}


@pytest.mark.parametrize("content,what", [
    ('{"letterMap": {"A": 1}, "substMap": {}}', "consecutive"),
    ('{"letterMap": {"A": 0, "R": 1}, "substMap": {"m": [1, 2, 3]}}', "2x2"),
    ('{"letterMap": {"A": 0}, "substMap": {"m": [1]}', "expected"),
])
def test_bad_subst_file(gsa_nw, tmp_path, content, what):
    sf = tmp_path / "subst.json"
    sf.write_text(content)
    r = run(gsa_nw, "-b", str(sf), "-r", os.path.join(RES, "param_best.json"), "-s",
            os.path.join(RES, "seq_generated.fa"), "--dryRun")
    assert r.returncode == 7 and what in r.stderr  # errorInvalidFormat


def test_bad_fasta_and_pairs(gsa_nw, tmp_path):
    fa = tmp_path / "s.fa"
    fa.write_text(">a\nARN\n>b\nAR#\n")
    r = run(gsa_nw, "-b", os.path.join(RES, "subst.json"), "-r", os.path.join(RES, "param_best.json"), "-s", str(fa),
            "--dryRun")
    assert r.returncode == 7 and ":4:3:" in r.stderr
    fa.write_text(">a\nARN\n>b\nARND\n")
    pf = tmp_path / "p.txt"
    pf.write_text("a b[2:9]\n")
    r = run(gsa_nw, "-b", os.path.join(RES, "subst.json"), "-r", os.path.join(RES, "param_best.json"), "-s", str(fa),
            "-p", str(pf), "--dryRun")
    assert r.returncode == 7 and "right bound" in r.stderr
    pf.write_text("a nosuch\n")
    r = run(gsa_nw, "-b", os.path.join(RES, "subst.json"), "-r", os.path.join(RES, "param_best.json"), "-s", str(fa),
            "-p", str(pf), "--dryRun")
    assert r.returncode == 7 and "unknown sequence id" in r.stderr


@pytest.mark.gpu
def test_known_answers_end_to_end(gsa_nw, tmp_path):
    """The reference's known answers through the reference's CLI: plain family (Gpu3 slot) is
    the source of truth, the sparse family (Gpu9 slot) must agree on cost, score hash and trace
    hash (else the driver exits with errorInvalidResult)."""
    known = json.load(open(os.path.join(ROOT, "tests", "golden", "known_answers.json")))
    pf = tmp_path / "pairs.txt"
    pf.write_text("".join(c["pair"] + "\n" for c in known["cases"][:5]))
    pj = tmp_path / "params.json"
    # the reference's slots with their param_best.json entries (every parameter they read is
    # required), this engine's slots with their own tile widths
    pj.write_text('{"NwAlign_Gpu3_Ml_DiagDiag": {"threadsPerBlockA": [96], "tileBx": [54]},'
                  ' "NwAlign_Gpu9_Mlsp_DiagDiagDiag": {"threadsPerBlockA": [128], "subtileRows": [4],'
                  ' "subtileCols": [4], "subtileBx": [48]},'
                  ' "NwAlign_Amd_Strip_Mlsp": {"tileBx": [256, 64]}, "NwAlign_Amd_Strip_Mlsppt": {"tileBx": [128]}}')
    out = tmp_path / "res.tsv"
    r = run(gsa_nw, "-b", os.path.join(RES, "subst.json"), "-r", str(pj), "-s", os.path.join(RES, "seq_generated.fa"),
            "-p", str(pf), "-o", str(out), "--fCalcScoreHash", "--fCalcTrace", "--warmupPerAlign", "1",
            "--samplesPerAlign", "2")
    assert r.returncode == 0, r.stderr
    rows = list(csv.DictReader(open(out), delimiter="\t"))
    assert len(rows) == 5 * 5
    by = {}
    for row in rows:
        assert row["err_step"] == "0" and row["nw_stat"] == "0"
        by.setdefault(row["seqY_id"] + " " + row["seqX_id"], []).append(row)
    for c in known["cases"][:5]:
        for row in by[c["pair"]]:
            assert int(row["align_cost"]) == c["align_cost"]
            assert row["score_hash"] == c["score_hash"]
            assert row["trace_hash"] == c["trace_hash"]
            if "edit_trace" in c:
                assert row["edit_trace"] == c["edit_trace"]
            assert float(row["align.calc"]) > 0
            # peak-alloc columns from the launch footprints (nwalign_shared.cpp:5-25)
            for col in ("glmem_peak_allocs", "shmem_peak_allocs", "regmem_peak_allocs"):
                assert int(row[col]) > 0, (col, row[col])
            assert int(row["locmem_peak_allocs"]) >= 0
