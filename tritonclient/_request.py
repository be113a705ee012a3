"""Outgoing-request view handed to plugins (reference tritonclient/_request.py:29-39)."""


class Request:
    """A request object whose ``headers`` dict plugins may edit."""

    def __init__(self, headers):
        self.headers = headers if headers is not None else {}
