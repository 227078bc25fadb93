import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(PKG_DIR, "build")


def lib_path(name):
    # SVO_LIB_DIR: a diagnostic build directory (e.g. build/stamps); libraries it lacks come from build/
    alt = os.environ.get("SVO_LIB_DIR")
    if alt and os.path.exists(os.path.join(alt, name)):
        return os.path.join(alt, name)
    return os.path.join(BUILD_DIR, name)
