"""Static check of the GPU-only Python entry points (bench.py, __graft_entry__,
scripts/): every name a function reads as a global must exist at module level
or in builtins.  These files run only on the GPU box, so an undefined name
would otherwise surface there first (no pyflakes in this image)."""
import builtins
import glob
import os
import symtable

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
FILES = [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")] + \
    sorted(glob.glob(os.path.join(ROOT, "scripts", "*.py")))


def undefined_globals(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols()
                    if s.is_assigned() or s.is_imported() or s.is_namespace()}
    known = module_names | set(dir(builtins)) | {"__file__", "__name__"}
    bad = []

    def walk(t):
        for s in t.get_symbols():
            if s.is_referenced() and s.is_global() and not s.is_declared_global() \
                    and s.get_name() not in known:
                bad.append(f"{t.get_name()}:{s.get_name()}")
        for c in t.get_children():
            walk(c)
    for c in top.get_children():
        walk(c)
    return bad


@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_no_undefined_globals(path):
    assert undefined_globals(path) == []
