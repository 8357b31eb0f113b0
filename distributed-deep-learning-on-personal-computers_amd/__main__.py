"""``python -m ddlpc ...`` -> :func:`ddlpc.cli.main`."""
import sys

from .cli import main

sys.exit(main())
