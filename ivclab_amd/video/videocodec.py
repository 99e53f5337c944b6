"""VideoCodec with the reference's interface (ivclab/video/videocodec.py:12-86), composed from
this package's GPU-backed parts: rgb2ycbcr / ycbcr2rgb (ivc_color.hip), IntraCodec (fused
DCT + quantisation + zig-zag + zero-run kernels), MotionCompensator (full-search ME and MC
kernels) and the host Huffman coder.

The reference's behaviour is kept as it is, quirks included:
  * frame 0 (I-frame) is IntraCodec.encode_decode of the luma plane with its 3-plane
    quantisation of a grayscale input, so the reconstruction is the first plane of a
    3-channel array (intracodec.py:109-138);
  * later frames (P-frames) raise ValueError, as the reference does: the motion-vector
    Huffman coder is trained on [-40, 40] for search_range 4 (videocodec.py:33, :58-60) but
    fed raster indices 0 .. (2sr+1)^2 - 1, so any index above 40 is "outside the trained
    range"; if every index fits, `prediction + recon_residual` adds an [H, W] array to the
    residual codec's [H, W, 3] reconstruction (videocodec.py:74) and NumPy's broadcasting
    fails.
Bitstreams and bit counts are those of this package's Huffman coder (the reference's
`constriction` trees are not available); reconstructions do not depend on them.
"""
from __future__ import annotations

import numpy as np

from ..entropy import HuffmanCoder
from ..image import IntraCodec
from ..signal.color import rgb2ycbcr, ycbcr2rgb
from .motion import MotionCompensator


class VideoCodec:

    def __init__(self, quantization_scale=1.0, bounds=(-1000, 4000), end_of_block=4000,
                 block_shape=(8, 8), search_range=4):
        """videocodec.py:14-35."""
        self.quantization_scale = quantization_scale
        self.bounds = bounds
        self.end_of_block = end_of_block
        self.block_shape = block_shape
        self.search_range = search_range
        self.intra_codec = IntraCodec(quantization_scale=quantization_scale, bounds=bounds,
                                      end_of_block=end_of_block, block_shape=block_shape)
        self.residual_codec = IntraCodec(quantization_scale=quantization_scale, bounds=bounds,
                                         end_of_block=end_of_block, block_shape=block_shape)
        self.motion_comp = MotionCompensator(search_range=search_range)
        self.motion_huffman = HuffmanCoder(lower_bound=-((2 * search_range + 1) ** 2 - 1) // 2)
        self.decoder_recon = None

    def encode_decode(self, frame, frame_num=0, is_source_rgb=False):
        """videocodec.py:37-86: (reconstructed uint8 RGB frame, bitstream, bit count)."""
        frame_ycbcr = rgb2ycbcr(frame.astype(np.float32))
        y = frame_ycbcr[..., 0]
        if frame_num == 0:
            self.intra_codec.train_huffman_from_image(y, is_source_rgb=False)
            recon_y, bitstream, residual_bits = self.intra_codec.encode_decode(y, is_source_rgb=False)
            motion_bits = 0
        else:
            ref_y = self.decoder_recon[..., 0] if self.decoder_recon.ndim == 3 else self.decoder_recon
            mv = self.motion_comp.compute_motion_vector(ref_y, y)
            flat_mv = mv.flatten()
            if frame_num == 1:
                n = (2 * self.motion_comp.search_range + 1) ** 2
                self.motion_huffman.train(np.full(n, 1.0 / n))
            mv_words, motion_bits = self.motion_huffman.encode(flat_mv)
            mv_dec = self.motion_huffman.decode(mv_words, len(flat_mv)).reshape(mv.shape)
            prediction = self.motion_comp.reconstruct_with_motion_vector(ref_y[..., np.newaxis],
                                                                         mv_dec)[..., 0]
            residual = y - prediction
            self.residual_codec.train_huffman_from_image(residual, is_source_rgb=False)
            recon_res, bitstream, residual_bits = self.residual_codec.encode_decode(
                residual, is_source_rgb=False)
            recon_y = prediction + recon_res
        self.decoder_recon = recon_y
        out = frame_ycbcr.copy()
        out[..., 0] = np.clip(recon_y[..., 0] if recon_y.ndim == 3 else recon_y, 0, 255)
        recon_rgb = ycbcr2rgb(out).astype(np.uint8)
        return recon_rgb, bitstream, residual_bits + motion_bits
