"""Import shim: makes the package directory `alpha-zero-general-inflexion_amd/`
importable as `azg_amd` (a hyphenated directory is not a valid module name)."""
import importlib.util as _ilu
import pathlib as _pl
import sys as _sys

_dir = _pl.Path(__file__).resolve().with_name("alpha-zero-general-inflexion_amd")
_spec = _ilu.spec_from_file_location(__name__, _dir / "__init__.py", submodule_search_locations=[str(_dir)])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
