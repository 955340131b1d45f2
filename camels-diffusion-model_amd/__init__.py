"""cdm_amd — MI355X-native (gfx950 HIP) ContextUnet DDPM for 64x64 CAMELS HI maps.

Drop-in for the reference's ContextUnet module API (ContextUnet.py), its diffusion helpers
(code/train_diffusion_condition.py) and the train_diffusion.py CLI.  Import as ``cdm_amd`` (the
repo-root ``cdm_amd.py`` shim maps the hyphenated directory to that name).
"""
from ._lib import lib  # noqa: F401
from .diffusion import DDPM, GraphSampler, Schedule, denoise_add_noise, perturb_input, sample_ddpm  # noqa: F401
from .likelihood import (LikelihoodEvaluator, calculate_elbo_and_bpd, calculate_elbo_and_bpd_batch,  # noqa: F401
                         calculate_elbo_and_bpd_dataset, calculate_likelihood)
from .model import ContextUnet, EmbedFC, ResidualConvBlock, UnetDown, UnetUp  # noqa: F401
from .stats import (calculate_power_spectrum_2d, compare_distributions, compare_power_spectra,  # noqa: F401
                    pdfs, power_spectra, power_spectrum)
from .trainer import Trainer  # noqa: F401

__all__ = ["ContextUnet", "EmbedFC", "ResidualConvBlock", "UnetDown", "UnetUp", "lib", "DDPM", "GraphSampler",
           "Schedule", "denoise_add_noise", "perturb_input", "sample_ddpm", "Trainer", "LikelihoodEvaluator",
           "calculate_likelihood", "calculate_elbo_and_bpd", "calculate_elbo_and_bpd_batch",
           "calculate_elbo_and_bpd_dataset", "power_spectrum", "power_spectra", "compare_power_spectra",
           "calculate_power_spectrum_2d", "compare_distributions", "pdfs"]
