"""compress_reconstruct — drop-in for engines/pipeline.py:17-167 of the reference.

One call = one jds_compress_reconstruct (include/jds.h): the image goes to the
MI355X once; the fused HIP kernels (csrc/jds_codec.hip) do colour conversion,
chroma prefilter + subsampling, reflect padding, 8x8 DCT, quantisation,
dequantisation, IDCT, chroma upsampling, colour conversion and truncation; the
same launch sequence accumulates the exact coefficient statistics, PSNR sums,
IntermediateData maps and the selected block, and K4 (csrc/jds_ssim.hip)
computes SSIM.  The host only builds the quantisation table and wraps results.
"""

from typing import Tuple

import numpy as np

from models.compression_params import CompressionParams
from models.compression_result import CompressionResult
from models.intermediate_data import IntermediateData
from engines.quantizer import scale_quant_matrix
from utils.constants import JPEG_LUMA_Q50
from utils.metrics import bitrate_from_counts, psnr_from_mse
from jds.codec import compress_reconstruct_raw


def compress_reconstruct(
    image_rgb: np.ndarray,
    params: CompressionParams,
    selected_block_idx: Tuple[int, int] = (0, 0)
) -> Tuple[CompressionResult, IntermediateData]:
    """Run the JPEG-like compression + reconstruction pipeline on the GPU."""
    if params.subsampling_mode not in ('4:4:4', '4:2:2', '4:2:0'):
        raise ValueError(f"Unknown subsampling mode: {params.subsampling_mode}")
    if params.block_size != 8:
        # the reference gets as far as quantize(), which broadcasts the BxB block
        # against the 8x8 table (engines/quantizer.py:24)
        b = params.block_size
        raise ValueError(f"operands could not be broadcast together with shapes ({b},{b}) (8,8) ")
    return _run(image_rgb, params, selected_block_idx)


def compress_reconstruct_stretch(
    image_rgb: np.ndarray,
    params: CompressionParams,
    selected_block_idx: Tuple[int, int] = (0, 0)
) -> Tuple[CompressionResult, IntermediateData]:
    """The same pipeline with block_size 8 or 16 (BASELINE configs[4] stretch).

    The reference accepts block_size=16 in CompressionParams but cannot run it;
    here 16x16 blocks use Q16 = np.kron(Q8, ones((2, 2))) (include/jds.h,
    DESIGN.md) with every other stage unchanged.  IntermediateData's
    selected_block_* fields are None for 16x16 blocks."""
    if params.subsampling_mode not in ('4:4:4', '4:2:2', '4:2:0'):
        raise ValueError(f"Unknown subsampling mode: {params.subsampling_mode}")
    if params.block_size not in (8, 16):
        b = params.block_size
        raise ValueError(f"operands could not be broadcast together with shapes ({b},{b}) (8,8) ")
    return _run(image_rgb, params, selected_block_idx)


def _run(image_rgb, params, selected_block_idx):
    q_matrix = scale_quant_matrix(JPEG_LUMA_Q50, params.quality)           # pipeline.py:43
    raw = compress_reconstruct_raw(image_rgb, params.quality, q_matrix, params.subsampling_mode,
                                   params.use_prefilter, params.block_size, selected_block_idx)
    st = raw['stats']
    h, w = raw['reconstructed'].shape[:2]
    if not (h >= 7 and w >= 7):
        # skimage.metrics.structural_similarity (utils/metrics.py:12-21)
        raise ValueError(
            "win_size exceeds image extent. Either ensure that your images are at least 7x7; or pass "
            "win_size explicitly in the function call, with an odd value less than or equal to the smaller "
            "side of your images. If your images are multichannel (with color channels), set channel_axis "
            "to the axis number corresponding to the channels.")

    ssim = np.ctypeslib.as_array(st.ssim).copy()
    bitrate = bitrate_from_counts(st.nonzero, st.magnitude_bits_f32, st.total_coeffs, (h, w),
                                  params.block_size)                        # pipeline.py:100
    result = CompressionResult(
        original_image=image_rgb,
        reconstructed_image=raw['reconstructed'],
        psnr_y=psnr_from_mse(st.mse_y),
        ssim_y=float(ssim[3]),
        psnr_rgb=psnr_from_mse(st.sse_rgb / (h * w * 3)),
        ssim_rgb=float(ssim[:3].mean()),
        bpp=bitrate['bpp'],
        compression_ratio=bitrate['compression_ratio'],
        nonzero_coeffs=bitrate['nonzero_count'],
        total_coeffs=bitrate['total_coeffs'],
        encode_time_ms=float(st.fwd_ms),
        decode_time_ms=float(st.inv_ms),
        bitrate_label=bitrate['label'],
    )
    sel = raw['selected'] or {}
    intermediate = IntermediateData(                                         # pipeline.py:153-165
        selected_block_idx=selected_block_idx,
        selected_block_original=sel.get('original'),
        selected_block_shifted=sel.get('shifted'),
        selected_block_dct=sel.get('dct'),
        selected_block_quantized=sel.get('quantized'),
        selected_block_dequantized=sel.get('dequantized'),
        selected_block_reconstructed=sel.get('reconstructed'),
        error_map_y=raw['error_map_y'],
        error_map_rgb=raw['error_map_rgb'],
        quantized_histogram=np.ctypeslib.as_array(st.hist).astype(np.int64),
        all_quantized_coeffs=raw['coeffs'],
    )
    return result, intermediate
