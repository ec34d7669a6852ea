"""``python -m fastapriori_amd <input> <output> [temp] [flags]`` — see fastapriori_amd/config.py."""
import sys

from .pipeline import main

if __name__ == "__main__":
    sys.exit(main())
