"""celestia_eds — MI355X-native extended-data-square hot path of celestia-app.

Python view of libcelestia_eds.so (HIP kernels for gfx950 + C ABI), with the
reference's package names: `da` (pkg/da), `wrapper` (pkg/wrapper), `rsmt2d`
(github.com/celestiaorg/rsmt2d), plus `device` for the device-resident batch API
used by bench.py.
"""
from . import _lib, da, rsmt2d, wrapper  # noqa: F401
from ._lib import CelError, Context, default_context, load  # noqa: F401
