from .frame import DKV, ENUM, INT, REAL, Frame, Vec  # noqa: F401
from .parse import import_file, parse_setup, parse_text  # noqa: F401
