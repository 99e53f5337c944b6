"""Host-code AddressSanitizer/UBSan driver (tests/test_asan_host.py runs it in a child process
with the clang ASan runtime preloaded).  It exercises, on the CPU only:
  * libivc's host C++ built with -fsanitize=address,undefined (--cuda-host-only): the
    Huffman coder (ivc_huffman.hip: code lengths, canonical encode/decode, every error
    path), and the argument checks / device-less failure paths of every C-ABI entry point;
  * the C oracle (oracle/ivc_oracle.c) built the same way: ME for every dtype and search
    range class, narrow/short frames, MC with out-of-frame indices.
Usage: python asan_driver.py <libivc_asan.so> <liboracle_asan.so>; exit 0 = clean."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def load_ivc(path):
    from ivclab_amd import _native as N
    L = C.CDLL(path)
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    return L


def huffman(L):
    rng = np.random.default_rng(0)
    cases = [np.array([1.0]), np.array([0.5, 0.5]), np.full(7, 1 / 7),
             rng.random(300) + 1e-9, np.geomspace(1, 1e-12, 64), rng.random(4096) ** 8 + 1e-12]
    for probs in cases:
        probs = np.ascontiguousarray(probs / probs.sum())
        n = probs.size
        lengths = np.zeros(n, np.uint8)
        assert L.ivc_huffman_lengths(ptr(probs), n, ptr(lengths)) == 0, L.ivc_last_error()
        lo = -n // 2
        sym = rng.integers(lo, lo + n, 5000).astype(np.int32)
        nbits = np.zeros(1, np.int64)
        cap = int(lengths.max()) * sym.size // 32 + 2
        words = np.zeros(cap, np.uint32)
        assert L.ivc_huffman_encode(ptr(sym), sym.size, lo, ptr(lengths), n, ptr(words), cap,
                                    ptr(nbits)) == 0, L.ivc_last_error()
        nw = (int(nbits[0]) + 31) // 32
        out = np.zeros(sym.size, np.int32)
        assert L.ivc_huffman_decode(ptr(words), nw, sym.size, lo, ptr(lengths), n, ptr(out)) == 0
        assert np.array_equal(out, sym)
        # too small a buffer, a symbol outside the alphabet, a truncated stream
        small = np.zeros(1, np.uint32)
        assert L.ivc_huffman_encode(ptr(sym), sym.size, lo, ptr(lengths), n, ptr(small), 1,
                                    ptr(nbits)) != 0 or sym.size * lengths.max() <= 32
        bad = sym.copy()
        bad[17] = lo + n
        assert L.ivc_huffman_encode(ptr(bad), bad.size, lo, ptr(lengths), n, ptr(words), cap,
                                    ptr(nbits)) != 0
        if nw > 1:
            L.ivc_huffman_decode(ptr(words), nw // 2, sym.size, lo, ptr(lengths), n, ptr(out))
    # invalid arguments
    z = np.zeros(4, np.float64)
    ln = np.zeros(4, np.uint8)
    assert L.ivc_huffman_lengths(ptr(z), 4, ptr(ln)) != 0           # non-positive weights
    assert L.ivc_huffman_lengths(None, 4, ptr(ln)) != 0
    assert L.ivc_huffman_lengths(ptr(z), -1, ptr(ln)) != 0
    assert L.ivc_huffman_decode(None, 1, 1, 0, ptr(ln), 4, None) != 0


def entry_point_errors(L):
    """Argument checks that return before any device work, and the no-device failures."""
    L.ivc_device_count()
    L.ivc_version()
    img = np.zeros((1, 16, 16, 1), np.uint8)
    tab = np.ones((3, 64), np.float64)
    q = np.zeros((1, 2, 2, 3, 64), np.int32)
    calls = [
        lambda: L.ivc_intra_encode(ptr(img), 1, 1, 15, 16, 1, ptr(tab), 10, 0, ptr(q)),   # H % 8
        lambda: L.ivc_intra_encode(ptr(img), 99, 1, 16, 16, 1, ptr(tab), 10, 0, ptr(q)),  # dtype
        lambda: L.ivc_intra_encode(None, 1, 1, 16, 16, 1, ptr(tab), 10, 0, ptr(q)),
        lambda: L.ivc_intra_encode(ptr(img), 1, -1, 16, 16, 1, ptr(tab), 10, 0, ptr(q)),
        lambda: L.ivc_intra_encode(ptr(img), 1, 1, 16, 16, 2, ptr(tab), 10, 0, ptr(q)),   # C = 2
        lambda: L.ivc_intra_encode(ptr(img), 1, 1, 16, 16, 1, ptr(tab), 10, 0, ptr(q)),   # no GPU
    ]
    a = np.zeros((16, 16), np.uint8)
    mv = np.zeros((2, 2), np.int64)
    calls += [
        lambda: L.ivc_motion_estimate(ptr(a), ptr(a), 1, 1, 16, 12, 4, 0, ptr(mv)),
        lambda: L.ivc_motion_estimate(ptr(a), ptr(a), 1, 1, 16, 16, -1, 0, ptr(mv)),
        lambda: L.ivc_motion_estimate(ptr(a), ptr(a), 42, 1, 16, 16, 4, 0, ptr(mv)),
        lambda: L.ivc_motion_estimate(ptr(a), ptr(a), 1, 1, 16, 16, 4, 7, ptr(mv)),
        lambda: L.ivc_motion_estimate(ptr(a), ptr(a), 1, 1, 16, 16, 4, 0, ptr(mv)),
    ]
    sym = np.zeros(128, np.int32)
    ns = np.zeros(1, np.int64)
    calls += [
        lambda: L.ivc_zerorun_encode(ptr(sym), 2, 64, 65, 4000, ptr(sym), 128, ptr(ns)),
        lambda: L.ivc_zerorun_encode(ptr(sym), -2, 64, 64, 4000, ptr(sym), 128, ptr(ns)),
        lambda: L.ivc_zerorun_decode(ptr(sym), 8, 2, 65, 4000, ptr(sym), ptr(ns)),
        lambda: L.ivc_zigzag(ptr(sym), 1, 64, 3, 0, ptr(sym)),
        lambda: L.ivc_zigzag(ptr(sym), 1, 32, 4, 1, ptr(sym)),
    ]
    for i, fn in enumerate(calls):
        rc = fn()
        assert rc != 0, f"call {i} unexpectedly succeeded"
        msg = L.ivc_last_error()
        assert msg, f"call {i}: empty error"


def oracle_c(path):
    O = C.CDLL(path)
    P, Lg, I = C.c_void_p, C.c_long, C.c_int
    O.oracle_me.argtypes = [P, P, I, I, Lg, Lg, I, Lg, Lg, P]
    O.oracle_me.restype = I
    O.oracle_mc.argtypes = [P, I, Lg, Lg, Lg, P, I, P]
    O.oracle_mc.restype = None
    dts = {"uint8": 1, "int8": 2, "uint16": 3, "int16": 4, "uint32": 5, "int32": 6,
           "uint64": 7, "int64": 8, "float32": 9, "float64": 10}
    rng = np.random.default_rng(1)
    for (H, W) in ((8, 8), (8, 224), (40, 16), (24, 40)):
        for name, code in dts.items():
            ref = rng.integers(0, 200, (H, W)).astype(name)
            cur = rng.integers(0, 200, (H, W)).astype(name)
            for sr in (0, 1, 4, 16, 23):
                mv = np.zeros((H // 8, W // 8), np.int64)
                assert O.oracle_me(ptr(ref), ptr(cur), code, 0, H, W, sr, 0, H // 8, ptr(mv)) == 0
                if name == "uint8":
                    mv2 = np.zeros_like(mv)
                    O.oracle_me(ptr(ref), ptr(cur), code, 1, H, W, sr, 1 if H > 8 else 0,
                                H // 8, ptr(mv2))
                for C_ in (1, 3):
                    img = rng.integers(0, 255, (H, W, C_)).astype(name)
                    idx = rng.integers(-5, (2 * sr + 1) ** 2 + 5, (H // 8, W // 8)).astype(np.int64)
                    out = np.zeros_like(img)
                    O.oracle_mc(ptr(img), img.itemsize, H, W, C_, ptr(idx), sr, ptr(out))


def main():
    ivc_so, oracle_so = sys.argv[1], sys.argv[2]
    L = load_ivc(ivc_so)
    huffman(L)
    entry_point_errors(L)
    oracle_c(oracle_so)
    print("asan driver: clean")


if __name__ == "__main__":
    main()
