"""Torch model definitions served by the bench server (random-init weights)."""
