"""CPU checks of bench.py (the driver runs it only on a GPU box): it imports, every global name
its functions load exists (a name lost in an edit otherwise shows up as a NameError on the
first GPU run), and its argument parser takes the documented workloads and flags."""
import builtins
import dis
import types

import pytest


def _code_objects(co):
    yield co
    for c in co.co_consts:
        if isinstance(c, types.CodeType):
            yield from _code_objects(c)


@pytest.mark.parametrize("module", ["bench", "__graft_entry__"])
def test_every_loaded_global_exists(module):
    mod = __import__(module)
    missing = set()
    for name, obj in vars(mod).items():
        if isinstance(obj, types.FunctionType) and obj.__module__ == module:
            for co in _code_objects(obj.__code__):
                for ins in dis.get_instructions(co):
                    if ins.opname == "LOAD_GLOBAL":
                        g = ins.argval
                        if g not in vars(mod) and not hasattr(builtins, g):
                            missing.add((name, g))
    assert not missing, sorted(missing)


def test_committed_traffic_summary_describes_these_kernels():
    """bench.py's roofline.traffic / frac_requests come from the committed PMC summary; it is
    used only when stamped with the digest of this tree's native sources (csrc + ABI header),
    so the committed file must carry that digest and the c5 probe's kernel (the mod-sampling
    instantiation at 6 proteins per block, annotate_kernel<8, 70, 6, true>) with its line
    requests, and bench.py's lookup resolves that record from the name it prints."""
    import json
    import bench
    import kmeranno
    d = json.load(open(bench.TRAFFIC_FILE))
    assert d["source_sha16"] == kmeranno.source_digest()
    rec = d["workloads"]["c5"]["annotate_kernel<8, 70, 6, true>"]
    assert rec["read_requests"] > 0 and rec["traffic_bytes"] > 0
    assert bench.kernel_capacity(8, "c5") == 6 and bench.kernel_capacity(8, "c4") == 4
    traffic, reqs, src, stale = bench.pmc_traffic("c5", "annotate_kernel<8, 70, *, true>")
    assert (traffic, reqs, stale) == (rec["traffic_bytes"], rec["read_requests"], False)
    for lf in ("0.75", "0.9"):
        assert f"c5_lf{lf}" in d["workloads"]
