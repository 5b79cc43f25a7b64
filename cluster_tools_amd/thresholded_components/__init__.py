from .thresholded_components_workflow import ThresholdedComponentsWorkflow  # noqa: F401
