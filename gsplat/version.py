from gaussctrl_exp_amd import __version__  # noqa: F401
