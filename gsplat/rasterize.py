"""gsplat 0.1.2.1 `gsplat.rasterize` module -> gaussctrl_exp_amd.rasterize (MI355X kernels)."""
import importlib

# importlib, not `import a.b as c`: the package attribute gaussctrl_exp_amd.rasterize may be a
# function of the same name.
_impl = importlib.import_module("gaussctrl_exp_amd.rasterize")

# re-export every public and private name (tests and callers reach e.g. _RasterizeGaussians)
globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
