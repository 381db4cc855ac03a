"""Install the witness engine as a Mythril plugin (entry point ``mythril.plugins``).

The native library is built in-tree (``python -m mythril_amd.build``) and shipped
as package data; see INTEGRATION.md.
"""
from setuptools import setup

setup(
    name="mythril-amd-witness",
    version="0.1.0",
    description="MI355X constraint-witness engine behind Mythril's get_model",
    packages=["mythril_amd"],
    # lib/asmjit_template.s: the assembled kernels' template (mythril_amd/asmjit.py);
    # csrc/*.inc: the generated asm interpreter the sources include
    package_data={"mythril_amd": ["lib/*.so", "lib/*.s", "csrc/*.h", "csrc/*.hip", "csrc/*.cpp", "csrc/*.inc"]},
    python_requires=">=3.8",
    install_requires=["numpy"],
    entry_points={"mythril.plugins": ["mi355x-witness-engine = mythril_amd.mythril_plugin:MI355XWitnessEngine"]},
)
