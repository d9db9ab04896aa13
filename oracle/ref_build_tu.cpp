// oracle/ref_build_tu.cpp — TEST INFRASTRUCTURE ONLY.
//
// Single translation unit that compiles the reference's own index builder
// (bowtie2-build-l) from the reference sources in place (-I/root/reference).
// The reference Makefile's bowtie2-build-l rule misses SHARED_CPPS,
// so we list the translation units it needs here.  No reference code is copied.
#include <utility>
#include <string>
#include <iostream>
using namespace std;
#include "ds.cpp"
#include "ccnt_lut.cpp"
#include "ref_read.cpp"
#include "alphabet.cpp"
#include "shmem.cpp"
#include "edit.cpp"
#include "bt2_locks.cpp"
#include "bt2_idx.cpp"
#include "bt2_io.cpp"
#include "bt2_util.cpp"
#include "reference.cpp"
#include "multikey_qsort.cpp"
#include "limit.cpp"
#include "random_source.cpp"
#include "diff_sample.cpp"
#include "bt2_build.cpp"
#include "bowtie_build_main.cpp"
