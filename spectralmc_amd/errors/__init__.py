"""Frozen error records with a ``kind`` tag (reference ``src/spectralmc/errors/``)."""
