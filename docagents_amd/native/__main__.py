import sys

from . import build

for k, v in build(force="--force" in sys.argv).items():
    print(k, v)
