"""The Erlang binding (nif/antidote_gpu_nif.c) cannot be built here (no
Erlang/OTP, no erl_nif.h); it is at least compiled for syntax and warnings
against the erl_nif API subset it uses (tests/nif_rt/erl_nif.h,
declarations only), and it must bind only symbols include/antidote_gpu.h
declares."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_nif_compiles_cleanly():
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "nif_rt"),
                        os.path.join(ROOT, "nif", "antidote_gpu_nif.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_nif_binds_declared_symbols_only():
    src = open(os.path.join(ROOT, "nif", "antidote_gpu_nif.c")).read()
    hdr = open(os.path.join(ROOT, "include", "antidote_gpu.h")).read()
    used = set(re.findall(r"\b(agn_[a-z_0-9]+)\s*\(", src))
    declared = set(re.findall(r"\b(agn_[a-z_0-9]+)\s*\(", hdr))
    assert used and used <= declared, used - declared
    # every engine-owned partition entry point of the drop-in is bound
    for f in ("agn_oplog_create", "agn_oplog_append", "agn_oplog_prune", "agn_oplog_destroy",
              "agn_batcher_create", "agn_batcher_create_cached", "agn_batcher_read",
              "agn_intern", "agn_materialize_host", "agn_gst_min"):
        assert f in used, f
