from oracle.pydp_restatement import create_partition_strategy  # noqa: F401


class PartitionSelectionStrategy:  # type name only
    pass
