"""The LDS-race guard, made deterministic (VERDICT r05 "next" #3).

Round 5 found `me_mfma16x2_kernel` reading a stale cross-wave `red[]` entry in ~4 % of cfg5
steps: hipcc emitted the loop-header `s_barrier` without an `s_waitcnt lgkmcnt(0)` while the
search's `red[]` writes from the back edge were still in flight.  The fix routes every device
barrier through `lds_barrier()` (ivc_internal.h: the wait, then the barrier).  These tests
check the *compiled* code, not the sources:

* `test_audit_flags_the_prefix_kernel` — the audit run on the committed pre-fix assembly
  (`tests/golden/me_mfma_a117a29_loop_header.s`: the a117a29 source compiled with the same
  flags) flags exactly the loop-header barrier;
* `test_every_compiled_barrier_drains_lds` — every `.hip` translation unit of libivc compiled
  to gfx950 assembly (hipcc -S, in parallel, ~1 min on this container's 8 cores): every
  `s_barrier` has an `s_waitcnt lgkmcnt(0)` after the last LDS instruction of its basic block.
"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from check_barriers import audit  # noqa: E402

from ivclab_amd import build as B  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "me_mfma_a117a29_loop_header.s")


def test_audit_flags_the_prefix_kernel():
    with open(FIXTURE) as f:
        asm = f.read()
    total, bad = audit(asm)
    assert total == 1 and len(bad) == 1
    lines = asm.split("\n")
    assert lines[bad[0] - 1].strip() == "s_barrier"
    # the red[] write the barrier fails to drain, and the merge read behind it
    assert any("ds_write_b64" in l and "offset:39008" in l for l in lines[:bad[0]])
    assert any("ds_read" in l and "offset:38912" in l for l in lines[bad[0]:])


def test_audit_accepts_a_drained_barrier():
    fixed = open(FIXTURE).read().replace("\ts_barrier", "\ts_waitcnt lgkmcnt(0)\n\ts_barrier")
    total, bad = audit(fixed)
    assert total == 1 and bad == []
    # a wait that an LDS instruction follows does not count
    late = open(FIXTURE).read().replace(
        "\ts_barrier", "\ts_waitcnt lgkmcnt(0)\n\tds_write_b32 v1, v2\n\ts_barrier")
    assert audit(late)[1]


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not present")
def test_every_compiled_barrier_drains_lds():
    flags = [f for f in B.FLAGS if f not in ("-shared", "-fPIC")]
    srcs = [s for s in B.SOURCES if s.endswith(".hip")]

    def one(src, d):
        out = os.path.join(d, src + ".s")
        subprocess.run([B.hipcc()] + flags + B.FILE_FLAGS.get(src, []) + ["-S", "--cuda-device-only", "-o", out,
                                              os.path.join(B.CSRC, src)],
                       check=True, capture_output=True, timeout=600)
        with open(out) as f:
            return src, audit(f.read())

    with tempfile.TemporaryDirectory() as d:
        with ThreadPoolExecutor(min(len(srcs), os.cpu_count() or 1)) as ex:
            res = dict(ex.map(lambda s: one(s, d), srcs))
    offenders = {s: bad for s, (_, bad) in res.items() if bad}
    assert not offenders, offenders
    # the kernels with LDS-sharing loops are all in there (a silent empty audit would pass)
    assert res["ivc_me_mfma.hip"][0] >= 4 and res["ivc_kernels.hip"][0] >= 100
    assert sum(t for t, _ in res.values()) >= 700
