"""Reference-compatible module tree (gfx950 backend: sfa_hip)."""
