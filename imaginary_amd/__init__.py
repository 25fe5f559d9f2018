"""imaginary_amd — MI355X-native pixel-transform engine for imaginary's hot path.

The product is libmipx.so (gfx950 HIP kernels + C-ABI, include/mipx.h); this
package is its Python binding plus a mirror of imaginary's operation layer.
Importing it fails when libmipx.so has not been built: there is no CPU path.
"""
from ._abi import lib, MipxError, MipxPlan, MipxOpts, MipxInput, LIB_PATH, TYPES, EXTEND, GRAVITY  # noqa: F401
from ._abi import (MIPX_OK, MIPX_EINVAL, MIPX_EUNSUPPORTED, MIPX_ENOMEM, MIPX_ENODEV, MIPX_EDEVICE,  # noqa: F401
                   MIPX_ETIMEOUT, MIPX_ENOTINIT, MIPX_ESTALE, MIPX_EBUSY)
from .engine import (DeviceBuffer, Engine, device_count, execute, fit_dimension, make_input,  # noqa: F401
                     make_opts, plan_chain, plan_make, reduce_sampling, run_op, set_reduce_sampling,
                     smartcrop_origins, synchronize)

__version__ = "0.2.0"
