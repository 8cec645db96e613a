"""setuptools entry: ``build_ext`` runs the in-tree hipcc builder.

    python setup.py build_ext --inplace   # == python -m agent_hypervisor_amd.utils.build
    pip install -e . --no-build-isolation

The extension (``agent_hypervisor_amd/_C*.so``) is compiled for gfx950 by
``agent_hypervisor_amd/utils/build.py`` (hipcc for csrc/host + csrc/hip, g++ for
csrc/cpu), not by setuptools' compiler abstraction.
"""

from setuptools import setup
from setuptools.command.build_ext import build_ext


class HipccBuild(build_ext):
    def run(self):
        from agent_hypervisor_amd.utils.build import build

        build(verbose=self.verbose)

    def get_outputs(self):
        from agent_hypervisor_amd.utils.build import ext_path

        return [str(ext_path())]


setup(cmdclass={"build_ext": HipccBuild})
