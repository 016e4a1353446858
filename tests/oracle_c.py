"""The C bit-model checker (oracle/stein_ref_c.py), under the name the tests import."""
from oracle.stein_ref_c import compact_ok, greedy, greedy_mt, greedy_ties, host_threads, lib, pairs, pow_15_25  # noqa: F401
