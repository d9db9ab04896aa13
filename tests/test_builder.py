"""bt2x_build_index (host C++ SA-IS builder) produces byte-identical .bt2l files to the
reference's bowtie2-build-l: checked against the committed reference-built indexes
(lambda = the reference's own example genome, rep = repeat-rich synthetic) and the md5s
of a FASTA exercising the record edge cases."""
import hashlib
import json
import lzma
import os

import pytest

import golden_io as g
from bt2x import lib


def md5(path):
    return hashlib.md5(open(path, "rb").read()).hexdigest()


@pytest.mark.parametrize("name,fasta", [("lambda_virus", None), ("rep", "rep.fa.xz")])
def test_builder_matches_reference_index(tmp_path, name, fasta):
    if fasta is None:
        # the reference's own example genome (example/reference/lambda_virus.fa, data file)
        fa = os.path.join(g.GOLDEN, "lambda_virus.fa")
    else:
        fa = str(tmp_path / "in.fa")
        with lzma.open(os.path.join(g.GOLDEN, fasta), "rb") as fi, open(fa, "wb") as fo:
            fo.write(fi.read())
    ref = g.materialize_index(name, str(tmp_path / "ref"))
    mine = lib.build_index(fa, str(tmp_path / "mine"))
    for k in "1234":
        assert md5(f"{mine}.{k}.bt2l") == md5(f"{ref}.{k}.bt2l"), k


def test_builder_record_edge_cases(tmp_path):
    exp = json.load(open(os.path.join(g.GOLDEN, "builder_md5.json")))["tricky"]
    mine = lib.build_index(os.path.join(g.GOLDEN, "tricky.fa"), str(tmp_path / "tricky"))
    for k in "1234":
        assert md5(f"{mine}.{k}.bt2l") == exp[k], k


def test_builder_with_supplied_sa(tmp_path):
    """bench.py's path: prefix-doubling SA (tools/gpu_sa.py, run on the CPU here) +
    bt2x_build_index_sa -> the same bytes as the reference-built rep index."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(g.HERE), "tools"))
    import gpu_sa
    import simdata as sd
    fa = str(tmp_path / "in.fa")
    with lzma.open(os.path.join(g.GOLDEN, "rep.fa.xz"), "rb") as fi, open(fa, "wb") as fo:
        fo.write(fi.read())
    codes, _ = sd.concat_genome(sd.read_fasta(fa))
    sa, bwt, keys = gpu_sa.suffix_array(codes[codes < 4], device="cpu")
    ref = g.materialize_index("rep", str(tmp_path / "ref"))
    mine = lib.build_index_sa(fa, str(tmp_path / "mine"), sa, bwt=bwt, keys=keys)
    for k in "1234":
        assert md5(f"{mine}.{k}.bt2l") == md5(f"{ref}.{k}.bt2l"), k
    # a corrupted SA is rejected
    bad = sa.copy()
    bad[-1] = 0
    with pytest.raises(lib.Bt2xError):
        lib.build_index_sa(fa, str(tmp_path / "bad"), bad)
