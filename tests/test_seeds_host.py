"""Host seed instantiation (bt2x/seeds.py) against the seeds the reference's
MultiSeedResults::instantiateSeeds produced for every golden read and round."""
import os
from collections import defaultdict

import numpy as np
import pytest

import golden_io as g
import seeds_ref as seeds


@pytest.mark.parametrize("fq,gold", [("lambda_longreads.fq.xz", "seeds_lambda.txt.xz"),
                                     ("rep_reads.fq.xz", "seeds_rep.txt.xz")])
def test_instantiation_matches_reference(fq, gold):
    reads = g.read_fastq(os.path.join(g.GOLDEN, fq))
    exp = defaultdict(list)
    with g.open_text(os.path.join(g.GOLDEN, gold)) as f:
        for line in f:
            if line.startswith("S "):
                t = [int(x) for x in line.split()[1:7]]
                exp[(t[0], t[1])].append((t[2], t[3], t[4], t[5]))
    got = {}
    for ri, (_, s, _) in enumerate(reads):
        c = g.codes(s)
        for r in range(2):
            lst = seeds.instantiate(c, 0, 0, r)
            if lst:
                got[(ri, r)] = [(int(fw), i, int(t[1]), int(t[2])) for fw, i, t in lst]
    assert set(got) == set(exp)
    for k in exp:
        assert got[k] == exp[k], k


def test_fixed_length_batch_matches_per_read():
    rng = np.random.default_rng(1)
    reads = rng.integers(0, 4, size=(50, 150)).astype(np.uint8)
    reads[3, 40] = 4
    buf, sin, ridx = seeds.batch_fixed_length(reads)
    per_read = []
    for k in range(len(reads)):
        for fw, i, t in seeds.instantiate(reads[k], 2 * k * 150, (2 * k + 1) * 150):
            per_read.append((t[0], t[1], t[2]))
    assert [(int(a), int(b), int(c)) for a, b, c in zip(sin["read_off"], sin["seed_off"], sin["seed_len"])] == per_read
    assert len(sin) == 50 * 18 - 2          # 9 seeds/strand at 150 bp; one N kills 1 fw + 1 rc
    np.testing.assert_array_equal(buf[150:300], np.where(reads[0] < 4, 3 - reads[0], 4)[::-1])
