"""TEST INFRASTRUCTURE — stand-in for python-dp, used ONLY to import the
reference (/root/reference) in the build container to generate golden vectors
(oracle/gen_golden.py).  Arithmetic lives in oracle/pydp_restatement.py."""
from . import _pydp  # noqa: F401
from . import algorithms  # noqa: F401
