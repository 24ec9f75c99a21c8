"""Import shim: the package directory is ``distributed-forecasting_amd/`` (the
layout the build spec names), which is not a valid Python identifier.  This
module makes it importable as ``distributed_forecasting_amd`` by pointing the
package search path at that directory and executing its ``__init__``."""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "distributed-forecasting_amd")]
__package__ = __name__
_init = _os.path.join(__path__[0], "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
