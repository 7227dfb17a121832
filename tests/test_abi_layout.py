"""The ctypes mirrors in porqua_amd/_lib.py against the C-ABI header: every struct's size and
the offset of its last field, from a C program compiled here with gcc against
include/porqua_hip.h (a layout drift would pass garbage to the kernels without any error)."""
import ctypes
import os
import shutil
import subprocess

import pytest

from porqua_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (C type, ctypes mirror, last field)
STRUCTS = [("pq_problem", _lib.PQProblem, "box_stride"), ("pq_state", _lib.PQState, "work_stride"),
           ("pq_settings", _lib.PQSettings, "min_iter"), ("pq_lowrank", _lib.PQLowRank, "dg_stride"),
           ("pq_gcap", _lib.PQGcap, None), ("pq_pg_wide", _lib.PQPgWide, "refine_steps")]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_ctypes_mirrors_match_the_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "porqua_hip.h"', 'int main(void) {']
    for cname, _, last in STRUCTS:
        off = f"offsetof({cname}, {last})" if last else "0"
        lines.append(f'  printf("%zu %zu\\n", sizeof({cname}), (size_t)({off}));')
    lines += ['  return 0;', '}']
    src = tmp_path / "abi.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for (cname, mirror, last), line in zip(STRUCTS, out):
        size, off = (int(v) for v in line.split())
        assert ctypes.sizeof(mirror) == size, (cname, ctypes.sizeof(mirror), size)
        if last:
            assert getattr(mirror, last).offset == off, (cname, last, getattr(mirror, last).offset, off)
