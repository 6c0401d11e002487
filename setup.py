"""Packaging (reference: Code/setup.py, ``packages=['cgnn']``): installs the drop-in
``cgnn`` package and the ``cgnn_amd`` framework.  The native extensions (HIP kernels
for gfx950 via hipcc, the host C++ runtime via g++) are built by ``cgnn_amd._build``
as the build_ext step:

    python setup.py build_ext --inplace      # in-tree build (what the tests use)
    pip install --no-build-isolation .       # installed copy
"""
import os
import sys

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(Command):
    description = "build the HIP (gfx950) and host C++ extensions with cgnn_amd._build"
    user_options = [("inplace", "i", "build in the source tree"), ("force", "f", "rebuild everything"),
                    ("debug", "g", "host runtime with ASan/UBSan")]
    boolean_options = ["inplace", "force", "debug"]

    def initialize_options(self):
        self.inplace = True
        self.force = False
        self.debug = False

    def finalize_options(self):
        pass

    def run(self):
        sys.path.insert(0, ROOT)
        from cgnn_amd import _build
        _build.build_all(force=bool(self.force), verbose=True, debug=bool(self.debug))


class BuildPyWithNative(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(
    name="cgnn_amd",
    version="2.0",
    description="Causal Generative Neural Networks (and a GNN training track) native to AMD MI355X",
    license="Apache-2.0",
    packages=find_packages(include=["cgnn", "cgnn.*", "cgnn_amd", "cgnn_amd.*"]),
    package_data={"cgnn_amd": ["*.so", "csrc/include/*.h", "csrc/kernels/*", "csrc/runtime/*"]},
    python_requires=">=3.8",
    install_requires=["numpy", "scipy", "pandas", "scikit-learn", "torch"],
    cmdclass={"build_ext": BuildNative, "build_py": BuildPyWithNative},
)
