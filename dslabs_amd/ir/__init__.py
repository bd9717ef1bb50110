"""Protocol IR (see core.py): declarative protocol descriptions that generate both the packed
device protocol and the oracle's object form."""
from .core import Protocol, lit, select  # noqa: F401
