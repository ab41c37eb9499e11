from .builder import (build_model, build_criterion_metrics, build_optimizer, wrap_model,  # noqa: F401
                      autocast_dtype, build_loader, pretune_model)
