"""HuffmanCoder with the reference's interface (ivclab/entropy/huffman.py:5-61), coded on
the host in libivc (ivc_huffman_*: the serial bit-packing stays on the host by design; the
GPU produces the symbols and their histogram).

The reference builds its trees with the `constriction` wheel, which is not available here;
this coder uses canonical Huffman codes with a deterministic tie-break.  Decoding its own
bitstreams is exact; bitstreams and (on messages that are not the training distribution)
bit counts are not pinned to the reference's.
"""
from __future__ import annotations

from itertools import combinations

import numpy as np

from .. import _native as N


class HuffmanCoder:
    def __init__(self, lower_bound=0):
        self.lower_bound = lower_bound
        self.probs = None
        self.encoder_codebook = None     # code lengths per symbol (canonical code)
        self.decoder_codebook = None

    def train(self, probs):
        """huffman.py:12-19."""
        probs = np.asarray(probs)
        if np.any(probs == 0):
            raise ValueError("Zero-probability symbols found in PMF. All symbols must have "
                             "non-zero probability.")
        self.probs = probs
        w = np.ascontiguousarray(probs, dtype=np.float64)
        lengths = np.zeros(max(w.size, 1), np.uint8)
        N.check(N.load_library().ivc_huffman_lengths(N.ptr(w), w.size, N.ptr(lengths)),
                "huffman")
        self.encoder_codebook = lengths[:w.size]
        self.decoder_codebook = self.encoder_codebook

    def encode(self, message):
        """huffman.py:21-34: (compressed words, number of bits)."""
        if self.encoder_codebook is None:
            raise RuntimeError("Train the Huffman coder before encoding.")
        message = np.asarray(message)
        max_symbol = len(self.probs) - 1 + self.lower_bound
        if np.any((message < self.lower_bound) | (message > max_symbol)):
            raise ValueError("Message contains symbols outside the trained range.")
        sym = np.ascontiguousarray(message.ravel(), dtype=np.int32)
        L = self.encoder_codebook
        cap = int((L[sym - self.lower_bound].astype(np.int64).sum() + 31) // 32) if sym.size else 0
        words = np.zeros(max(cap, 1), np.uint32)
        nbits = np.zeros(1, np.int64)
        N.check(N.load_library().ivc_huffman_encode(N.ptr(sym), sym.size, int(self.lower_bound),
                                                    N.ptr(L), L.size, N.ptr(words), cap,
                                                    N.ptr(nbits)), "huffman_encode")
        return words[:cap], float(nbits[0])

    def decode(self, compressed, message_length):
        """huffman.py:36-45."""
        if self.decoder_codebook is None:
            raise RuntimeError("Train the Huffman coder before decoding.")
        words = np.ascontiguousarray(compressed, dtype=np.uint32)
        out = np.empty(max(int(message_length), 1), np.int32)
        L = self.decoder_codebook
        N.check(N.load_library().ivc_huffman_decode(N.ptr(words), words.size, int(message_length),
                                                    int(self.lower_bound), N.ptr(L), L.size,
                                                    N.ptr(out)), "huffman_decode")
        return np.asarray(out[:int(message_length)].astype(np.int64))

    def code_of(self, i):
        """The canonical code of symbol index i as a list of bits."""
        L = self.encoder_codebook
        order = np.lexsort((np.arange(L.size), L))
        code, prev = 0, 0
        for j, s in enumerate(order):
            if j:
                code = (code + 1) << (int(L[s]) - prev)
            prev = int(L[s])
            if s == i:
                return [(code >> k) & 1 for k in range(prev - 1, -1, -1)]
        raise IndexError(i)

    def is_prefix_free(self):
        """huffman.py:47-53."""
        codes = ["".join(map(str, self.code_of(i))) for i in range(len(self.probs))]
        for a, b in combinations(codes, 2):
            if a.startswith(b) or b.startswith(a):
                return False
        return True
