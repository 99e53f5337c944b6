from .io import imread, imshow  # noqa: F401
from .metrics import calc_mse, calc_psnr  # noqa: F401
from .shape import Patcher, ZigZag  # noqa: F401
