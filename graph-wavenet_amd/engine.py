"""Drop-in for the reference's ``engine.py`` (``from engine import trainer``)."""
from gwn_amd.engine import FlatAdam, trainer  # noqa: F401
