"""Client plugin interface (reference tritonclient/_plugin.py:31-48)."""
from abc import ABC, abstractmethod


class InferenceServerClientPlugin(ABC):
    """Base class of every client plugin.

    A plugin is a callable applied to each outgoing :class:`Request` before it
    hits the network; it must mutate ``request.headers`` in place.
    """

    @abstractmethod
    def __call__(self, request):
        """Mutate ``request`` (a :class:`tritonclient.Request`) in place."""
