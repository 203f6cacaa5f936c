"""Register the package directory `recommender-system-using-apache-spark-mllib-_amd/`
under the importable name `als_mi355x` (the directory name has hyphens)."""
import importlib.util
import os
import sys

PKG_NAME = "als_mi355x"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "recommender-system-using-apache-spark-mllib-_amd")


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
