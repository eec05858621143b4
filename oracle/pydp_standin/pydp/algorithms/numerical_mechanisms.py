from oracle.pydp_restatement import GaussianMechanism, LaplaceMechanism  # noqa: F401
