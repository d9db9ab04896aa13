"""bench.py's harness on CPU: the CPU-baseline sample and the parity comparison under the
driver's step split (a sample larger than one step file), and the N>1 path under
torch.distributed.run (gloo, world size 2) with the host driver over the CPU oracle
kernels as the aligner (tests/cpp/test_e2e_oracle, bt2x-align's command line)."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
import bench  # noqa: E402

ORACLE_DRIVER = os.path.join(ROOT, "tests", "cpp", "test_e2e_oracle")


def _fq(path, first, n):
    with open(path, "w") as f:
        for i in range(first, first + n):
            f.write(f"@r{i}\nACGT\n+\nIIII\n")


def test_head_fastq_spans_step_files(tmp_path):
    # the driver's --steps 20 makes step files of 500 k reads, smaller than the 800 k sample
    files = [str(tmp_path / f"s{k}.fq") for k in range(3)]
    for k, p in enumerate(files):
        _fq(p, 5 * k, 5)
    dst = str(tmp_path / "sample.fq")
    assert bench.head_fastq(files, dst, 8) == 8
    assert open(dst).read().split("\n")[0::4][:8] == [f"@r{i}" for i in range(8)]
    assert bench.head_fastq(files, dst, 100) == 15                 # the stream is shorter
    assert bench.head_fastq(files[0], dst, 3) == 3


def test_parity_compares_the_same_reads(tmp_path):
    ours, ref = tmp_path / "ours.sam", tmp_path / "ref.sam"
    recs = [f"r{i}\t0\tchr\t{i}\t42" for i in range(10)]
    ours.write_text("@HD\tVN:1.0\n" + "".join(r + "\n" for r in recs))
    ref.write_text("@HD\tVN:1.0\n" + "".join(r + "\n" for r in reversed(recs[:6])))
    p = bench.parity(str(ours), str(ref), 6)
    assert p["records_differ"] == 0 and p["records_ours"] == p["records_reference"] == 6
    ref.write_text("".join(r + "\n" for r in recs[:5]) + "r5\t16\tchr\t5\t42\n")
    assert bench.parity(str(ours), str(ref), 6)["records_differ"] == 1


def test_host_threads_split_is_reported():
    class A:
        host_threads = 0
    t, note = bench.host_threads(A(), 128, 8)
    assert t == 16 and "below" not in note
    t, note = bench.host_threads(A(), 16, 8)
    assert t == 2 and "host-bound" in note
    A.host_threads = 5
    assert bench.host_threads(A(), 16, 8) == (5, "set by --host-threads")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_on_cpu(tmp_path):
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run, one process per
    rank): per-rank inputs, rank 0 indexes while rank 1 waits at the barrier, both align
    after a barrier, the counters are summed and the time is the max over ranks; rank 0
    prints one JSON line whose value counts both ranks' reads."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", BT2X_BENCH_DIR=str(tmp_path / "work"))
    reads = 1200
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--reads", str(reads), "--genome-mb", "0.25",
           "--replay-reads", "200", "--slots", "512", "--host-threads", "2", "--no-replay", "--no-cpu",
           "--cpu-index", "--aligner", ORACLE_DRIVER, "--runs", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "weak"
    e = line["end_to_end"]
    assert e["summary"][0] == f"{2 * reads} reads; of these:"
    assert abs(line["value"] - 2 * reads / e["t_align_max_s"] / 1e6) < 1e-3
    assert e["t_align_max_s"] >= e["t_align_s"] > 0
    assert line["config"]["host_threads"] == 2
    # two timed runs, each over both ranks; value is the median (here: the slower) run's
    assert len(e["runs"]) == 2 and all(x["value"] > 0 for x in e["runs"])
    assert any(abs(x["t_align_max_s"] - e["t_align_max_s"]) < 1e-3 for x in e["runs"])
    assert e["reaped_at_exit"] == []


def test_bench_eight_ranks_on_cpu(tmp_path):
    """bench.py --gpus 8 as the driver launches it on an 8-GPU node (torch.distributed.run,
    gloo, one process per rank), the host driver over the CPU oracle as the aligner: the
    counters sum to all ranks' reads, every rank ran on its own CPUs (the aligners report
    their affinity; the sets are disjoint and inside this process's), the threads per rank
    are the CPU share split 8 ways, and the note says when that leaves a rank host-bound."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", BT2X_BENCH_DIR=str(tmp_path / "work"))
    reads = 600
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--reads", str(reads), "--genome-mb", "0.25",
           "--replay-reads", "200", "--slots", "512", "--no-replay", "--no-cpu",
           "--cpu-index", "--aligner", ORACLE_DRIVER, "--runs", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8
    e, cfg = line["end_to_end"], line["config"]
    assert e["summary"][0] == f"{8 * reads} reads; of these:"
    assert abs(line["value"] - 8 * reads / e["t_align_max_s"] / 1e6) < 1e-3
    share = bench.cpu_share()
    assert cfg["host_threads"] == max(1, share // 8)
    assert cfg["host_threads_note"].startswith(f"{share}-CPU share / 8 rank(s)")
    if share // 8 < 14:
        assert "host-bound" in cfg["host_threads_note"]
    from bt2x import dist as bdist
    sets = [set(bdist.parse_cpu_list(c)) for c in cfg["host_cpus"]]
    assert len(sets) == 8 and all(sets)
    allowed = os.sched_getaffinity(0)
    assert all(s <= allowed for s in sets)
    for i in range(8):
        for j in range(i + 1, 8):
            assert not (sets[i] & sets[j]), (i, j, cfg["host_cpus"])
    assert cfg["host_cpus_note"]


def test_rank_cpu_sets_split_each_gpu_node():
    """The per-rank CPU sets on an 8-GPU, 2-socket node: four ranks per socket, each a
    disjoint slice of whole cores (SMT siblings together) of its GPU's NUMA node; a GPU
    with no known node draws from the CPUs left over."""
    from bt2x import dist as bdist
    node = {0: list(range(0, 64)) + list(range(128, 192)), 1: list(range(64, 128)) + list(range(192, 256))}
    core = {c: c % 128 for c in range(256)}
    sets, note = bdist.rank_cpu_sets(list(range(8)), range(256), [0, 0, 0, 0, 1, 1, 1, 1], node, core)
    assert [bdist.format_cpu_list(s) for s in sets] == [
        "0-15,128-143", "16-31,144-159", "32-47,160-175", "48-63,176-191",
        "64-79,192-207", "80-95,208-223", "96-111,224-239", "112-127,240-255"]
    assert "node0: 4 rank(s) x 32 CPUs" in note
    # a cgroup cpuset that leaves part of each node, and one GPU of unknown node
    allowed = list(range(0, 32)) + list(range(64, 96))
    sets, note = bdist.rank_cpu_sets([0, 1, 2], allowed, [0, 1, -1], node, core)
    assert sets[0] == list(range(0, 32)) and sets[1] == list(range(64, 96)) and sets[2] == allowed
    # (no CPU left over for the unknown-node rank: it shares the allowed set, and says so)
    assert "no NUMA split" in note
    assert bdist.parse_cpu_list("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_bench_one_rank_with_config_legs_on_cpu(tmp_path):
    """bench.py at N=1 with the C2 (E. coli, --no-sse8) and C5 (400 bp) legs, at toy sizes,
    through the host driver over the CPU oracle: every leg reports a rate, C5 aligns nothing
    (reads of 256 bp or more), and the reference baselines and parity run where the
    reference binaries are built."""
    env = dict(os.environ, OMP_NUM_THREADS="2", BT2X_BENCH_DIR=str(tmp_path / "work"))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--reads", "600",
           "--genome-mb", "0.25", "--replay-reads", "200", "--slots", "512", "--host-threads", "2", "--no-replay",
           "--cpu-index", "--aligner", ORACLE_DRIVER, "--c2-reads", "1500", "--c5-reads", "1000",
           "--cpu-sample", "300", "--cpu-sample-1t", "100", "--no-rep-leg", "--runs", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    legs = line["configs_other"]
    assert legs["C2"]["reads"] == 1500 and legs["C2"]["value"] > 0 and legs["C2"]["aligned"] > 1400
    assert legs["C5"]["reads"] == 900 and legs["C5"]["aligned"] == 0          # the first file is untimed
    if os.access(os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l"), os.X_OK):
        assert line["parity"]["records_differ"] == 0 and line["parity"]["sample_reads"] == 300
        assert legs["C2"]["parity"]["records_differ"] == 0 and legs["C5"]["parity"]["records_differ"] == 0


def test_bench_repeat_leg_on_cpu(tmp_path):
    """The optional repeat-heavy sensitivity leg (--rep-leg) at toy size through the host
    driver over the CPU oracle: a rate, the DP work per read field (bt2x-align --stats), and (where the reference binary is
    built) its baseline and 0 differing records."""
    env = dict(os.environ, OMP_NUM_THREADS="2", BT2X_BENCH_DIR=str(tmp_path / "work"))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--reads", "400",
           "--genome-mb", "0.25", "--replay-reads", "200", "--slots", "512", "--host-threads", "2", "--no-replay",
           "--cpu-index", "--aligner", ORACLE_DRIVER, "--no-legs", "--no-cpu", "--rep-leg", "--rep-mb", "0.3",
           "--rep-reads", "1500"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    leg = line["configs_other"]["C3_rep50"]
    assert leg["reads"] == 1500 and leg["value"] > 0 and leg["aligned"] > 1000 and "dps_per_read" in leg
