"""Kernel resource usage of the built library (CPU test, reads the compiler's remarks).

kmers.anno_amd/Makefile compiles every device object with -Rpass-analysis=kernel-resource-usage
into build/*.o.res. A kernel of ours that uses scratch (private) memory is a regression: in
round 3 a select over a register array was folded into a dynamically indexed private copy,
annotate_kernel<8, 6, 8> took 48 bytes per lane of scratch and c5 wrote ~2.2 GB of it per
launch (profiles/r03_traffic.json of the r03i pass). Library kernels (rocPRIM's sorts) are not ours.
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "kmers.anno_amd", "build")


def kernel_usage():
    out = {}
    for f in sorted(glob.glob(os.path.join(BUILD, "*.o.res"))):
        name = None
        for line in open(f, errors="replace"):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                out[name] = {}
                continue
            m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[", line)
            if m and name:
                out[name][m.group(1).strip()] = int(m.group(2))
    return out


@pytest.fixture(scope="module")
def usage():
    u = kernel_usage()
    if not u:
        pytest.skip("no build/*.o.res (build the library with kmers.anno_amd/Makefile)")
    return u


def test_no_scratch_in_our_kernels(usage):
    ours = {k: v for k, v in usage.items() if "rocprim" not in k}
    assert len(ours) > 50
    bad = {k: v.get("ScratchSize") for k, v in ours.items() if v.get("ScratchSize", 0) != 0}
    assert not bad, f"kernels with scratch memory: {bad}"


def test_hot_kernels_occupancy(usage):
    # the protein probe keeps 7 waves per SIMD (amdgpu_waves_per_eu(7, 8)); the 6-frame probe 7
    # (its four sequential 256-position slices per block, KMA_CONTIG_SEQ; 8 with one)
    hot = {"annotate_kernelILi8ELi6ELi8E": 7, "contigs_probe_quad_kernelILi8ELi6E": 7}
    for frag, occ in hot.items():
        names = [k for k in usage if frag in k]
        assert names, frag
        for k in names:
            assert usage[k]["Occupancy"] >= occ, (k, usage[k])
