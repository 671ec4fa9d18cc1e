"""Search pipelines: the MI355X BRP search and its numerical references."""
from .search import BRPSearch, SearchConfig, SearchOutput, app_binary  # noqa: F401
from .multi import MultiWUSearch  # noqa: F401
from . import reference  # noqa: F401
