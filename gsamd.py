"""Import shim: the package directory is `gelly-streaming_amd/` (not a Python
identifier). `import gsamd` loads it as the module `gelly_streaming_amd` and
returns it; submodules (e.g. `gelly_streaming_amd.distributed`) resolve normally."""
import importlib.util
import os
import sys

_NAME = "gelly_streaming_amd"
_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gelly-streaming_amd")

if _NAME in sys.modules:
    _mod = sys.modules[_NAME]
else:
    _spec = importlib.util.spec_from_file_location(_NAME, os.path.join(_DIR, "__init__.py"),
                                                   submodule_search_locations=[_DIR])
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules[_NAME] = _mod
    _spec.loader.exec_module(_mod)

sys.modules[__name__] = _mod
