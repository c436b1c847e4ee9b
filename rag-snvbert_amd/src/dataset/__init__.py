"""Featurisation, panel data and retrieval datasets (reference: src/dataset/)."""
