"""Post-fit utilities around the VI loop."""
from .alignment import (align_latent_positions, align_signs, align_temporal_states,
                        compute_alignment_error, compute_correlation_after_alignment,
                        procrustes_alignment)
from .diagnostics import compare_methods, compute_state_prediction_error
from .timing import run_method_with_timing

__all__ = ["procrustes_alignment", "align_signs", "align_latent_positions",
           "align_temporal_states", "compute_alignment_error",
           "compute_correlation_after_alignment", "compare_methods",
           "compute_state_prediction_error", "run_method_with_timing"]
