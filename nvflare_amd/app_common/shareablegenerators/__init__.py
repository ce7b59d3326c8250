from .full_model_shareable_generator import FullModelShareableGenerator, apply_weight_diff  # noqa: F401
