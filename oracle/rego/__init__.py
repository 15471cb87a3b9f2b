"""Rego subset interpreter (oracle; test infrastructure only)."""
from .interp import Interpreter  # noqa: F401
from .parser import parse_module  # noqa: F401
from .values import NULL, Arr, Num, Obj, RegoError, RSet, from_json_text, from_py, term_string, to_py  # noqa: F401
