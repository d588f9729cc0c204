from .quant import fp8_amax, fp8_dequantize, fp8_quantize  # noqa: F401
from .reduce import reduce, reduce_host  # noqa: F401
