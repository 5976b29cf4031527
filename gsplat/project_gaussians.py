"""gsplat 0.1.2.1 `gsplat.project_gaussians` module -> gaussctrl_exp_amd.project_gaussians (MI355X kernels)."""
import gaussctrl_exp_amd.project_gaussians as _impl

# re-export every public and private name (tests and callers reach e.g. _RasterizeGaussians)
globals().update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
