"""Train loop mirror of src/runner (trainers resolvable by name, main.py:99)."""
from . import trainers  # noqa: F401
