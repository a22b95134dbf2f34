"""interpolation-engine_amd: MI355X-native `{key}` interpolation (the hot path of
tillfalko/interpolation-engine), HIP kernels behind the C ABI of include/ie_amd.h.

Import this directory as the package `interpolation_engine_amd` (its on-disk name has a hyphen):
see __graft_entry__.load_package().
"""
from . import _native  # noqa: F401
from .interpolation_engine import (  # noqa: F401
    InsertsTable,
    InsertsTableSet,
    InterpolationException,
    VersionedInserts,
    display_text,
    display_texts,
    ingest_args,
    ingest_user_input,
    ingest_user_inputs,
    get_interpdata,
    get_simple_insertkey,
    interpolate_batch,
    interpolate_inserts,
    interpolate_states,
    recursive_escape,
    recursive_interpolate,
    recursive_interpolate_states,
    recursive_unescape,
    unescape_command,
)
from .maps import goto_map, goto_map_states, replace_map, replace_map_states  # noqa: F401
from .multi import MultiDevice, shard_bounds  # noqa: F401
from .wildcard import Wildcards, get_wildcard_matches, is_wildcard_match  # noqa: F401

__version__ = "0.1.0"
