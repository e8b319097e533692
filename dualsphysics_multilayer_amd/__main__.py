"""``python -m dualsphysics_multilayer_amd <case> <dirout> [options]`` — run a case (run.py)."""
import sys

from .run import main

sys.exit(main())
