"""Build hook of the installable package (pyproject.toml): compile the native libraries
in-tree (fastapriori_amd/ops/build.py: g++ for libfa_host.so, hipcc --offload-arch=gfx950
for libfa_hip.so) before the package files are collected, so the wheel carries them.
An installed copy has no csrc/ next to it: its libraries are loaded as shipped
(ops/_native.py records their build ids instead of checking them against sources)."""
import importlib.util
import os

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_py):
    def run(self):
        # ops/build.py by path: importing the package would import torch and the models
        spec = importlib.util.spec_from_file_location("fa_native_build",
                                                      os.path.join(ROOT, "fastapriori_amd", "ops", "build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        host, hip = mod.build_all(force=False)
        print(f"native libraries: {host}, {hip}")
        super().run()


class BinaryDistribution(Distribution):
    """The wheel carries native libraries: a platform wheel, not a pure-Python one."""

    def has_ext_modules(self):
        return True


setup(
    name="fastapriori_amd",
    version="0.1.0",
    description="MI355X-native frequent-itemset miner and association-rule recommender "
                "(FastApriori capabilities on HIP/CDNA4 + RCCL)",
    license="GPL-3.0-or-later",
    python_requires=">=3.10",
    install_requires=["torch", "numpy"],
    packages=["fastapriori_amd", "fastapriori_amd.models", "fastapriori_amd.ops", "fastapriori_amd.parallel",
              "fastapriori_amd.utils"],
    package_data={"fastapriori_amd.ops": ["*.so"]},
    entry_points={"console_scripts": ["fastapriori = fastapriori_amd.pipeline:main"]},
    cmdclass={"build_py": BuildNative},
    distclass=BinaryDistribution,
)
