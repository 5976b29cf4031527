"""gsplat 0.1.2.1 `gsplat.utils` module -> gaussctrl_exp_amd.utils (MI355X kernels)."""
import importlib

# importlib, not `import a.b as c`: the package attribute gaussctrl_exp_amd.utils may be a
# function of the same name.
_impl = importlib.import_module("gaussctrl_exp_amd.utils")

# re-export every public and private name (tests and callers reach e.g. _RasterizeGaussians)
globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
