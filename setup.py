"""Packaging for jax_llama_amd (reference ``setup.py:6`` packages ``jax_llama`` 0.0.0).

``pip install -e .`` / ``python setup.py build_ext --inplace`` compile the native extensions for
gfx950 through ``build.py`` (hipcc ``--offload-arch=gfx950``; the HIP kernels + torch bindings as
``jax_llama_amd/_C*.so`` and the Llama-3 BPE core as ``jax_llama_amd/_bpe*.so``) and ship them
next to the Python package, so the runtime never JIT-compiles anything.
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_ext):
    """Runs build.py (incremental, in-tree) instead of setuptools' compiler drivers."""

    def run(self):
        sys.path.insert(0, ROOT)
        import build as native_build
        for out in native_build.build_all(jobs=min(8, os.cpu_count() or 4)):
            print("built", out)


class BuildPyWithNative(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(
    name="jax_llama_amd",
    version="0.1.0",
    description="MI355X-native (gfx950) LLaMA-1/2/3 inference with the LSaldyt/JAX_llama API",
    packages=find_packages(include=["jax_llama_amd", "jax_llama_amd.*"]),
    package_data={"jax_llama_amd": ["_C*.so", "_bpe*.so", "csrc/**/*", "ops/tune_*.json"]},
    include_package_data=True,
    python_requires=">=3.10",
    install_requires=["torch", "numpy", "sentencepiece", "regex"],
    cmdclass={"build_ext": BuildNative, "build_py": BuildPyWithNative},
    zip_safe=False,
)
