"""Reference-compatible ``config`` package (gfx950 backend: sfa_hip).

Modules of the reference's ``config/`` that this drop-in does not provide resolve to the
reference's own files (sfa_hip/dropin.py: the package path falls through to every
reference sfa root on sys.path / in SFA_REFERENCE_ROOT).
"""

from sfa_hip import dropin as _dropin

__path__ = _dropin.package_path(__path__, __name__)
