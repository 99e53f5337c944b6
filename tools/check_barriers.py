"""Every s_barrier of the gfx950 code objects has an s_waitcnt lgkmcnt(0) in front of it in its
basic block (ivc_internal.h lds_barrier: hipcc leaves the wait out at some loop-header
barriers, and another wave can then read LDS as it was before a write).
Compiles each device source to assembly (about a minute) and lists offenders.
    python tools/check_barriers.py"""
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ivclab_amd import build as B  # noqa: E402


def audit(asm):
    lines, bad, total = asm.split("\n"), [], 0
    for i, l in enumerate(lines):
        if not l.strip().startswith("s_barrier"):
            continue
        total += 1
        j = i - 1
        while j >= 0:
            t = lines[j].strip()
            if re.match(r"^\.?LBB\w*:", t) or t.startswith("; %bb") or t.startswith("ds_"):
                bad.append(i + 1)
                break
            if t.startswith("s_waitcnt") and "lgkmcnt(0)" in t:
                break
            j -= 1
    return total, bad


def one(src, out):
    flags = [f for f in B.FLAGS if f not in ("-shared", "-fPIC")]
    subprocess.run([B.hipcc()] + flags + B.FILE_FLAGS.get(src, []) + ["-S", "--cuda-device-only", "-o", out,
                                          os.path.join(B.CSRC, src)], check=True,
                   capture_output=True)
    with open(out) as f:
        return src, audit(f.read())


def main():
    with tempfile.TemporaryDirectory() as d:
        srcs = [s for s in B.SOURCES if s.endswith(".hip")]
        with ThreadPoolExecutor(len(srcs)) as ex:
            res = list(ex.map(lambda s: one(s, os.path.join(d, s + ".s")), srcs))
    nbad = 0
    for src, (total, bad) in res:
        print(f"{src}: {total} barriers, {len(bad)} without lgkmcnt(0)" + (f" at lines {bad[:8]}" if bad else ""))
        nbad += len(bad)
    sys.exit(1 if nbad else 0)


if __name__ == "__main__":
    main()
