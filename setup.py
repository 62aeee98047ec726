"""Packaging shim: ``pip install .`` / ``python setup.py build_ext --inplace`` compile the native
module with hipcc for gfx950 through ``ddlb_amd._build`` (no hipify, no cpp_extension)."""

from setuptools import setup
from setuptools.command.build_ext import build_ext
from setuptools.dist import Distribution


class HipBuild(build_ext):
    def run(self):
        from ddlb_amd import _build

        _build.build()

    def get_outputs(self):
        from ddlb_amd import _build

        return [_build.ext_path()]


class BinaryDistribution(Distribution):
    def has_ext_modules(self):
        return True


setup(cmdclass={"build_ext": HipBuild}, distclass=BinaryDistribution)
