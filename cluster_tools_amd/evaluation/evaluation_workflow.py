"""EvaluationWorkflow (reference: cluster_tools/evaluation/evaluation_workflow.py:46-84): same
parameters (seg_path / seg_key / gt_path / gt_key / output_path / ignore_label).  The reference
chains NodeLabelWorkflow (overlaps) -> Measures; on the MI355X the overlaps and the measures are
one device pass, so the DAG is the single Measures task.  target must be 'local'."""
from cluster_tools_amd.luigi_compat import Parameter, BoolParameter
from cluster_tools_amd.cluster_tasks import WorkflowBase
from cluster_tools_amd.evaluation import measures as measure_tasks


class EvaluationWorkflow(WorkflowBase):
    seg_path = Parameter()
    seg_key = Parameter()
    gt_path = Parameter()
    gt_key = Parameter()
    output_path = Parameter()
    ignore_label = BoolParameter(default=True)

    def requires(self):
        measure_task = getattr(measure_tasks, self._get_task_name('Measures'))
        return measure_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                            seg_path=self.seg_path, seg_key=self.seg_key, gt_path=self.gt_path,
                            gt_key=self.gt_key, output_path=self.output_path, ignore_label=self.ignore_label,
                            dependency=self.dependency)

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'measures': measure_tasks.MeasuresLocal.default_task_config()})
        return configs
