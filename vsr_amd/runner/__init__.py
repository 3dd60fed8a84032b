"""Train / test loop mirror of src/runner (trainers and predictors resolvable by name, main.py:99,113)."""
from . import predictors, trainers  # noqa: F401
