"""dtype / device / optimiser-state models of the public API (reference ``src/spectralmc/models/``)."""
