"""dslabs_amd: MI355X-native breadth-first model checking for DSLabs protocols.

The product is ``libdslabs_hip.so`` (HIP kernels for gfx950 behind the C ABI in
include/dslabs_hip.h); this package is the thin host-side mirror of the reference's
``Search`` / ``SearchSettings`` / ``SearchResults`` API over it.
"""
from .search import (CLIENTS_DONE, NONE_DECIDED, RESULTS_OK, EndCondition, Engine, PredicateResult,  # noqa: F401
                     Search, SearchResults, SearchSettings, SearchState, StatePredicate, clientDone,
                     clientHasResults)

__all__ = ["Search", "SearchSettings", "SearchState", "SearchResults", "EndCondition", "StatePredicate",
           "PredicateResult", "Engine", "RESULTS_OK", "CLIENTS_DONE", "NONE_DECIDED", "clientDone",
           "clientHasResults"]
