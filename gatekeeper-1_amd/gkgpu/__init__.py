"""gkgpu — Python binding of libgkgpu.so (MI355X batch policy-evaluation engine).

``Driver`` mirrors the constraint framework's ``drivers.Driver`` plugin
interface (vendor/github.com/open-policy-agent/frameworks/constraint/pkg/
client/drivers/interface.go:21-39) over the C ABI in include/gkgpu.h.
``Client`` (client.py) mirrors the frameworks ``Client`` calls that reach the
driver, so tests and the bench exercise the same boundary a cgo shim would.

There is no CPU evaluation path in this package: if the native library or a
HIP device is missing, evaluation raises ``EngineUnavailable``.
"""
from .driver import Driver, EngineUnavailable, QueryError, Results, lib_path, load_library  # noqa: F401
from .client import Client, TARGET  # noqa: F401
