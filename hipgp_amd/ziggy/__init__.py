"""MI355X mirror of the reference `ziggy` package API for the Toeplitz/PCG hot path."""
