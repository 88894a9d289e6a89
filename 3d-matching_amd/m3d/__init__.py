"""m3d — MI355X-native (gfx950) point-cloud registration core.

Host layer (Python, ctypes) over libm3d.so, the HIP kernels behind the C ABI of
``include/m3d.h``.  See DESIGN.md for the path, the data layout and the kernels.
"""

from . import _lib, synth  # noqa: F401
from .types import PointCloud, RegistrationResult  # noqa: F401

__version__ = "0.1.0"


def library_path() -> str:
    return str(_lib.LIB_PATH)
