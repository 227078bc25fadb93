import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(PKG_DIR, "build")


def lib_path(name):
    return os.path.join(BUILD_DIR, name)
