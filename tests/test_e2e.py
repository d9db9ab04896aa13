"""End-to-end parity: FASTQ in, SAM out, against the reference aligner's own SAM.

Goldens (tests/golden/e2e_*.sam.xz) are the output of the reference's bowtie2-align-l
(1 thread) on the committed lambda and rep fixtures, as sorted, @PG-less records
(tools/make_golden.py e2e; the reference's own comparison methodology, scripts/sim
Sim.pm).  Sets: the lambda example reads (2000 records, 40-2561 bp, most unaligned by
the fork's length limits), and 3660 rep reads of 12-160 bp (repeats, N runs, indels)
under the default scoring, --dpad 12 and a non-default scoring scheme; the tandem-repeat
set; the i16 kernel's sets (the -DENABLE_I16 reference build); and, as md5s of the
sorted records (e2e_md5.json), all 6000 lambda reads (config C1), the 4.64 Mbp E. coli
stand-in (config C2, u8 and i16) and 50k x 150 bp reads (lane-kernel DP launches).

* `-m "not gpu"`: tests/cpp/test_e2e_oracle — the product's host driver
  (omp-bowtie2-prime_amd/host: per-read coroutine, prioritizeSATups, extendSeeds,
  reporting, MAPQ, SAM, the F11 edit-buffer replay) with the CPU oracle standing in for
  the three kernels.  This pins the host logic without a GPU.
* `-m gpu`: the product binary bt2x-align (host driver over libbt2x.so, every seed
  search / SA resolution / DP on the MI355X).
"""
from __future__ import annotations

import hashlib
import json
import lzma
import os
import subprocess

import pytest

import golden_io as g

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALIGN = os.path.join(ROOT, "omp-bowtie2-prime_amd", "bt2x", "bt2x-align")
ORACLE_DRIVER = os.path.join(ROOT, "tests", "cpp", "test_e2e_oracle")
ALT_OPTS = ["--mp", "5,1", "--np", "2", "--rdg", "4,2", "--rfg", "6,3", "--gbar", "2"]
WIDE_MIN = ["--score-min", "L,-0.6,-2.5", "--dpad", "12"]
# (name, index, reads, options): goldens from bowtie2-align-l; the *_i16 sets from the
# -DENABLE_I16 build bowtie2-align-l-i16 (tools/make_golden.py i16): --no-sse8 runs the
# signed 16-bit DP (config C2's kernel); "mix" is that build's default, where only reads
# whose minimum score falls below -254 take the i16 kernel (bt2x-align --i16-build)
SETS = [("e2e_lambda", "lambda_virus", "lambda_longreads.fq", []),
        ("e2e_rep", "rep", "rep_reads.fq", []),
        ("e2e_rep_dpad12", "rep", "rep_reads.fq", ["--dpad", "12"]),
        ("e2e_rep_alt", "rep", "rep_reads.fq", ALT_OPTS),
        ("e2e_tandem", "tandem", "tandem_reads.fq", []),
        ("e2e_tandem_dpad12", "tandem", "tandem_reads.fq", ["--dpad", "12"]),
        ("e2e_rep_i16", "rep", "rep_reads.fq", ["--no-sse8"]),
        ("e2e_tandem_i16", "tandem", "tandem_reads.fq", ["--no-sse8"]),
        ("e2e_rep_i16_wide", "rep", "rep_reads.fq", ["--no-sse8"] + WIDE_MIN),
        ("e2e_rep_i16_mix", "rep", "rep_reads.fq", ["--i16-build"] + WIDE_MIN)]
# the DP kernel modes each set runs through on the GPU: the launcher's default
# (lane-per-problem banded kernel above BT2X_DP_WAVE_MAX problems, wave per problem
# below), and each kernel forced for every launch
DP_MODES = {"default": None, "lane": "0", "wave": "1", "hostwin": "host", "handover": "handover", "parwave": "parwave",
            "stream2": "stream2", "lane1": "lane1", "split": "split", "nostore": "nostore", "wavefull": "wavefull", "gpusam": "gpusam"}
MD5 = os.path.join(g.GOLDEN, "e2e_md5.json")
SUMMARY = os.path.join(g.GOLDEN, "e2e_summary.json")


def split_stderr(text: str) -> tuple[list[str], str]:
    """(sorted per-read warning lines, the alignment summary block) of an aligner's stderr:
    the reference prints both (printEEScoreMsg, AlnSink::printAlSumm)."""
    lines = text.splitlines()
    warns = sorted(ln for ln in lines if ln.startswith("Warning:"))
    start = next((i for i, ln in enumerate(lines) if ln.endswith(" reads; of these:") or ln.endswith(" reads")), None)
    assert start is not None, "no alignment summary in:\n" + text[-1500:]
    end = next(i for i in range(start, len(lines)) if lines[i].endswith("overall alignment rate"))
    return warns, "".join(ln + "\n" for ln in lines[start:end + 1])


def check_summary(stderr: bytes, name: str) -> None:
    """The run's summary and warnings == the reference's (e2e_summary.json, make_golden.py summary)."""
    with open(SUMMARY) as f:
        exp = json.load(f)["sets"][name]["summary"]
    got_w, got_s = split_stderr(stderr.decode())
    exp_w, exp_s = split_stderr(exp)
    assert got_s == exp_s, f"summary:\n{got_s}\nreference:\n{exp_s}"
    assert got_w == exp_w, f"{len(got_w)} warnings vs the reference's {len(exp_w)}"


def sam_records(data: bytes) -> list[bytes]:
    lines = [ln for ln in data.split(b"\n") if ln and not ln.startswith(b"@PG")]
    return [ln for ln in lines if ln.startswith(b"@")] + sorted(ln for ln in lines if not ln.startswith(b"@"))


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory):
    d = tmp_path_factory.mktemp("e2e")
    out = {}
    for _, idx, fq, _ in SETS:
        if idx not in out:
            out[idx] = g.materialize_index(idx, str(d))
        if fq not in out:
            p = d / fq
            with lzma.open(os.path.join(g.GOLDEN, fq + ".xz"), "rb") as fi:
                p.write_bytes(fi.read())
            out[fq] = str(p)
    return out


def check(cmd: list[str], golden: str, env=None):
    r = subprocess.run(cmd, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    got = sam_records(r.stdout)
    with lzma.open(os.path.join(g.GOLDEN, golden + ".sam.xz"), "rb") as f:
        exp = sam_records(f.read())
    bad = [(a, b) for a, b in zip(got, exp) if a != b]
    assert len(got) == len(exp) and not bad, \
        f"{len(bad)} of {len(exp)} records differ; first:\n ours {bad[0][0][:300]!r}\n ref  {bad[0][1][:300]!r}" \
        if bad else f"{len(got)} records vs {len(exp)}"
    return got, r.stderr


@pytest.mark.parametrize("name,idx,fq,opts", SETS, ids=[s[0] for s in SETS])
def test_host_driver_vs_reference_sam(fixtures, name, idx, fq, opts):
    """Host driver + CPU oracle kernels == the reference's SAM (no GPU)."""
    assert os.access(ORACLE_DRIVER, os.X_OK), "build first: make -C tests/cpp"
    got, err = check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4", "--metrics"] + opts, name)
    check_summary(err, name)
    n_al = sum(1 for ln in got if not ln.startswith(b"@") and ln.split(b"\t")[1] != b"4")
    # (150 bp reads need --dpad <= 12 to fit ALN_MAX_COLS: SURVEY F2)
    assert n_al > {"lambda_virus": 400, "rep": 2000, "tandem": 1400}[idx]
    if name.startswith("e2e_rep_i16"):
        # the i16 kernel's RNG reseed (aligner_sw.cpp:338-348) changes records vs the u8 run
        with lzma.open(os.path.join(g.GOLDEN, "e2e_rep.sam.xz"), "rb") as f:
            assert sum(1 for a, b in zip(got, sam_records(f.read())) if a != b) > 20
    if idx == "tandem":
        # the fixture's point: -M tightens minsc between nextAlignment calls of one DP
        # problem (records consumed after a tightening in the same problem)
        tight = int(err.split(b"tight_recs=")[1].split()[0])
        assert tight > 100, tight


@pytest.mark.parametrize("name,idx,fq,opts", [SETS[1], SETS[9]], ids=[SETS[1][0], SETS[9][0]])
def test_host_driver_host_cut_windows(fixtures, name, idx, fq, opts):
    """The same with the DP reference windows cut by the driver (RefInfo::stretch) instead of
    named for the backend to cut (BT2X_DP_REF_TEXT, the GPU backend's default)."""
    check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4", "--host-windows"] + opts, name)


@pytest.mark.parametrize("name,idx,fq,opts", [SETS[1], SETS[4]], ids=[SETS[1][0], SETS[4][0]])
def test_host_driver_vs_reference_sam_three_requests(fixtures, name, idx, fq, opts):
    """The same with every seed round as seed search + host ranking/prioritization + SA
    resolution (the path a read takes when the GPU round hands it back)."""
    check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4", "--no-gpu-round"] + opts, name)


@pytest.mark.parametrize("name,idx,fq,opts", [SETS[1], SETS[4]], ids=[SETS[1][0], SETS[4][0]])
def test_host_driver_two_backends(fixtures, name, idx, fq, opts):
    """The same with the second cohort's launches on a backend of its own (bt2x-align's
    second context, bt2x_open_shared): two GPU threads whose launches overlap."""
    check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4", "--streams", "2"] + opts, name)


@pytest.mark.parametrize("mode", ["pipeline", "two", "serial"])
def test_host_driver_backend_error_exits_cleanly(fixtures, mode):
    """A backend failure (a GPU call's bt2x::Error) on a pipelined GPU thread reaches the
    caller as an exception: exit code 1 and the message, not std::terminate (SIGABRT)."""
    cmd = [ORACLE_DRIVER, fixtures["rep"], fixtures["rep_reads.fq"], "--slots", "400", "-p", "3",
           "--inject-error", "3"] + {"pipeline": [], "two": ["--streams", "2"], "serial": ["--no-pipeline"]}[mode]
    r = subprocess.run(cmd, capture_output=True, timeout=600)
    assert r.returncode == 1, (r.returncode, r.stderr[-500:])
    assert b"injected backend error" in r.stderr


def test_host_driver_slot_count_invariance(fixtures):
    """Results do not depend on how many reads are in flight."""
    outs = []
    for slots in ("1", "64", "5000"):
        r = subprocess.run([ORACLE_DRIVER, fixtures["rep"], fixtures["rep_reads.fq"], "--slots", slots, "-p", "3"],
                           capture_output=True, timeout=600, check=True)
        outs.append(sam_records(r.stdout))
    assert outs[0] == outs[1] == outs[2]


GPU_CASES = [(s, m) for s in SETS for m in DP_MODES
             if m == "default" or (m in ("hostwin", "handover") and s[0] in ("e2e_rep", "e2e_rep_i16_mix"))
             or (m == "parwave" and s[0] in ("e2e_rep", "e2e_tandem", "e2e_tandem_i16", "e2e_rep_i16_mix"))
             or (m in ("lane1", "split") and s[0] in ("e2e_rep", "e2e_rep_dpad12", "e2e_tandem"))
             or (m in ("nostore", "stream2", "gpusam") and s[0] in ("e2e_rep", "e2e_rep_i16_mix", "e2e_tandem"))
             or (m == "wavefull" and s[0] in ("e2e_rep", "e2e_rep_dpad12", "e2e_tandem_i16"))
             or (m in ("lane", "wave") and s[0] in ("e2e_rep", "e2e_rep_dpad12", "e2e_tandem", "e2e_rep_i16",
                                                    "e2e_tandem_i16", "e2e_rep_i16_mix"))]


@pytest.mark.gpu
@pytest.mark.parametrize("case,mode", GPU_CASES, ids=[f"{c[0]}-{m}" for c, m in GPU_CASES])
def test_bt2x_align_vs_reference_sam(fixtures, case, mode):
    """The product binary (kernels on the MI355X) == the reference's SAM, through each DP
    kernel: the launcher's choice, the banded lane kernels (lane: the launcher's lane
    choice; lane1: one lane per problem; split: the two-wave split fill) / the wave kernel
    forced (wave: its banded traceback layout, the default; wavefull: whole rectangles), the
    mismatch-only records' tails formatted on the GPU (gpusam: bt2x_sam_tails; by default the
    host formats every record), and the lane kernel handing nearly every walk over to the wave kernel (a 2-step
    budget)."""
    name, idx, fq, opts = case
    env = dict(os.environ)
    env.pop("BT2X_DP_WAVE", None)
    env.pop("BT2X_HOST_WINDOWS", None)
    env.pop("BT2X_DP_HEAVY", None)
    env.pop("BT2X_DP_PARWALK", None)
    env.pop("BT2X_DP_DUO", None)
    env.pop("BT2X_DP_SPLIT", None)
    env.pop("BT2X_READ_STORE", None)
    env.pop("BT2X_DP_WAVE_BAND", None)
    env.pop("BT2X_GPU_SAM", None)
    if DP_MODES[mode] == "host":
        env["BT2X_HOST_WINDOWS"] = "1"          # DP windows cut on the host (RefInfo::stretch)
    elif DP_MODES[mode] == "handover":
        env["BT2X_DP_WAVE"] = "0"
        env["BT2X_DP_HEAVY"] = "2"
    elif DP_MODES[mode] == "parwave":             # wave per problem, its parallel walk
        env["BT2X_DP_WAVE"] = "1"
        env["BT2X_DP_PARWALK"] = "2"
    elif DP_MODES[mode] == "lane1":               # lane kernels, one lane per problem (dp_fill_kernel)
        env["BT2X_DP_WAVE"] = "0"
        env["BT2X_DP_DUO"] = "0"
    elif DP_MODES[mode] == "split":               # lane kernels: the two-wave split fill (dp_split_kernel)
        env["BT2X_DP_WAVE"] = "0"
        env["BT2X_DP_SPLIT"] = "1"
    elif DP_MODES[mode] == "wavefull":            # wave per problem, whole rectangles in LDS
        env["BT2X_DP_WAVE"] = "1"
        env["BT2X_DP_WAVE_BAND"] = "0"
    elif DP_MODES[mode] == "gpusam":              # mismatch-only records' tails from bt2x_sam_tails
        env["BT2X_GPU_SAM"] = "1"
    elif DP_MODES[mode] == "nostore":             # reads sent with every request (no read store)
        env["BT2X_READ_STORE"] = "0"
    elif DP_MODES[mode] not in (None, "stream2"):
        env["BT2X_DP_WAVE"] = DP_MODES[mode]
    # stream2: the two cohorts on two contexts (bt2x_open_shared); default: one context
    env.pop("BT2X_STREAMS", None)
    extra = ["--streams", "2"] if DP_MODES[mode] == "stream2" else []
    _, err = check([ALIGN, "-x", fixtures[idx], "-U", fixtures[fq], "--slots", "1000"] + opts + extra, name, env=env)
    check_summary(err, name)


# ---------------------------------------------------------------- md5 goldens
# Sets too large to commit as SAM (tests/golden/e2e_md5.json, tools/make_golden.py md5):
# config C1 whole (6000 lambda reads; SURVEY.md:508's md5), config C2 (the seeded 4.64 Mbp
# E. coli stand-in, 10k x 100 bp, u8 and i16), and 50k x 150 bp at --dpad 12 whose DP
# launches exceed 32k problems (the banded lane kernel, end to end).

def md5_sets():
    with open(MD5) as f:
        return json.load(f)


def sam_md5(data: bytes) -> tuple[str, int]:
    lines = [ln for ln in data.split(b"\n") if ln and not ln.startswith(b"@PG")]
    recs = [ln for ln in lines if not ln.startswith(b"@")]
    return hashlib.md5(b"".join(ln + b"\n" for ln in sorted(lines))).hexdigest(), len(recs)


@pytest.fixture(scope="module")
def ecoli(tmp_path_factory):
    """The C2 genome stand-in indexed by bt2x_build_index, checked byte for byte against the
    reference builder's index (md5s in e2e_md5.json)."""
    import simdata as sd
    from bt2x import lib
    meta = md5_sets()
    d = tmp_path_factory.mktemp("ecoli")
    fa = str(d / "ecoli.fa")
    sd.write_fasta(fa, sd.ecoli_genome())
    assert hashlib.md5(open(fa, "rb").read()).hexdigest() == meta["ecoli_fasta_md5"]
    base = lib.build_index(fa, str(d / "ecoli"))
    for k, h in meta["ecoli_index_md5"].items():
        assert hashlib.md5(open(f"{base}.{k}.bt2l", "rb").read()).hexdigest() == h, k
    reads = {}
    for name, st in meta["sets"].items():
        if st["genome"] == "ecoli":
            path = str(d / f"{name}.fq")
            sd.fixture_reads(sd.ecoli_genome(), path, st["reads"], st["read_len"], st["seed"])
            reads[name] = path
    return base, reads


def lambda_full(tmp_path) -> str:
    p = tmp_path / "longreads.fq"
    with lzma.open(os.path.join(g.GOLDEN, "lambda_longreads_full.fq.xz"), "rb") as fi:
        p.write_bytes(fi.read())
    return str(p)


def check_md5(cmd: list[str], name: str, env=None):
    st = md5_sets()["sets"][name]
    r = subprocess.run(cmd, capture_output=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    h, n = sam_md5(r.stdout)
    assert (h, n) == (st["md5"], st["records"]), f"{name}: md5 {h} of {n} records != {st['md5']} of {st['records']}"
    return r.stderr


def md5_opts(st) -> list[str]:
    return [o for o in st["opts"]]


@pytest.mark.parametrize("name", ["ecoli_u8", "ecoli_i16", "ecoli_c5_400", "ecoli_long_200"])
def test_host_driver_vs_reference_md5_ecoli(ecoli, name):
    """Config C2 (u8 and the i16 kernel) and config C5's 400 bp reads (and 200 bp ones): host
    driver + CPU oracle kernels == reference."""
    base, reads = ecoli
    err = check_md5([ORACLE_DRIVER, base, reads[name], "--slots", "2000", "-p", "4", "--metrics"]
                    + md5_opts(md5_sets()["sets"][name]), name)
    check_summary(err, name)


def test_host_driver_vs_reference_md5_lambda_full(tmp_path):
    """Config C1, all 6000 reads (SURVEY.md:508: md5 1a34e0b9bc4cba5eef64e4ac8eb034c0)."""
    assert md5_sets()["sets"]["lambda_full"]["md5"] == "1a34e0b9bc4cba5eef64e4ac8eb034c0"
    base = g.materialize_index("lambda_virus", str(tmp_path))
    check_md5([ORACLE_DRIVER, base, lambda_full(tmp_path), "--slots", "777", "-p", "4"], "lambda_full")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ecoli_u8", "ecoli_i16", "ecoli_large_u8", "ecoli_large_i16", "ecoli_c5_400",
                                  "ecoli_long_200"])
def test_bt2x_align_vs_reference_md5_ecoli(ecoli, name):
    """Config C2, the 50k-read sets and config C5's fixed-length 400 bp reads (every record
    unaligned: reads of 256 bp or more never reach the seed search, bt2_search.cpp:2475-2496)
    on the MI355X.  The large sets run with every read in flight (--slots 65536): DP launches
    of more than 32k problems take the banded lane kernel (checked from the run's launch
    statistics)."""
    base, reads = ecoli
    large = "large" in name
    err = check_md5([ALIGN, "-x", base, "-U", reads[name], "--slots", "65536" if large else "4096", "--stats"]
                    + md5_opts(md5_sets()["sets"][name]), name)
    check_summary(err, name)
    if large:
        mx = int(err.split(b"dp_max_launch=")[1].split()[0])
        assert mx > 32768, mx


@pytest.mark.gpu
def test_bt2x_align_vs_reference_md5_lambda_full(tmp_path):
    base = g.materialize_index("lambda_virus", str(tmp_path))
    check_md5([ALIGN, "-x", base, "-U", lambda_full(tmp_path), "--slots", "1000"], "lambda_full")


def test_host_driver_lookahead_invariance(fixtures):
    """DP lookahead (problems posed ahead of need and memoised by DpKey) changes the
    number of launches, never the records."""
    outs = []
    for la in ("1", "8", "64"):
        r = subprocess.run([ORACLE_DRIVER, fixtures["rep"], fixtures["rep_reads.fq"], "--slots", "3000", "-p", "3",
                            "--dpad", "12", "--lookahead", la], capture_output=True, timeout=600, check=True)
        outs.append(sam_records(r.stdout))
    assert outs[0] == outs[1] == outs[2]
    with lzma.open(os.path.join(g.GOLDEN, "e2e_rep_dpad12.sam.xz"), "rb") as f:
        assert outs[0] == sam_records(f.read())


@pytest.mark.gpu
def test_bt2x_align_mates_align_as_unpaired(fixtures, tmp_path):
    """-1/-2 (config C4): this fork aligns mate 1 alone, as unpaired reads -- the
    records and summary of `-1 m1 -2 m2` equal those of `-U m1` (the reference's, measured:
    tools/make_golden.py; here the rep golden)."""
    m2 = tmp_path / "m2.fq"
    m2.write_bytes(open(fixtures["rep_reads.fq"], "rb").read())
    _, err = check([ALIGN, "-x", fixtures["rep"], "-1", fixtures["rep_reads.fq"], "-2", str(m2), "--slots", "1000"],
                   "e2e_rep")
    check_summary(err, "e2e_rep")
    r = subprocess.run([ALIGN, "-x", fixtures["rep"], "-1", fixtures["rep_reads.fq"], "-2", f"{m2},{m2}"],
                       capture_output=True, timeout=120)
    assert r.returncode == 1 and b"specified with -1, but 2" in r.stderr
