"""Authentication plugins."""
from ..._auth import BasicAuth

__all__ = ["BasicAuth"]
