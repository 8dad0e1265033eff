"""Window-LP export (native builder) and input preparation for the batched solver."""
from .builder import WindowGroup, battery_group, evaluate_terms, group_window_lps, pack_groups  # noqa: F401
