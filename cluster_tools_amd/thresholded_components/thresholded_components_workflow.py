"""ThresholdedComponentsWorkflow (reference: cluster_tools/thresholded_components/
thresholded_components_workflow.py:17-104): the same parameters and five-task DAG
(BlockComponents -> MergeOffsets -> BlockFaces -> MergeAssignments -> Write, in place, with
tmp/cc_offsets.json).  BlockComponents runs fused on the MI355X; the other tasks emit the
reference's artefacts.  target must be 'local'.

ThresholdAndWatershedWorkflow (thresholded_components_workflow.py:107-144): the components, then
WatershedFromSeeds with them as seeds, in place in the output dataset."""
import os

from cluster_tools_amd.luigi_compat import Parameter, FloatParameter, BoolParameter
from cluster_tools_amd.cluster_tasks import WorkflowBase
import cluster_tools_amd.utils.volume_utils as vu
from cluster_tools_amd.write import write as write_tasks
from cluster_tools_amd.thresholded_components import block_components as block_tasks
from cluster_tools_amd.thresholded_components import merge_offsets as offset_tasks
from cluster_tools_amd.thresholded_components import block_faces as face_tasks
from cluster_tools_amd.thresholded_components import merge_assignments as assignment_tasks
from cluster_tools_amd.watershed import watershed_from_seeds as ws_tasks


class ThresholdedComponentsWorkflow(WorkflowBase):
    input_path = Parameter()
    input_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    assignment_key = Parameter()
    threshold = FloatParameter()
    threshold_mode = Parameter(default='greater')
    mask_path = Parameter(default='')
    mask_key = Parameter(default='')
    channel = Parameter(default=None)
    fused = BoolParameter(default=True)

    def requires(self):
        block_task = getattr(block_tasks, self._get_task_name('BlockComponents'))
        offset_task = getattr(offset_tasks, self._get_task_name('MergeOffsets'))
        face_task = getattr(face_tasks, self._get_task_name('BlockFaces'))
        assignment_task = getattr(assignment_tasks, self._get_task_name('MergeAssignments'))
        write_task = getattr(write_tasks, self._get_task_name('Write'))
        with vu.file_reader(self.input_path, 'r') as f:
            shape = list(f[self.input_key].shape)
        if self.channel is None:
            assert len(shape) == 3
        else:
            assert len(shape) == 4
            shape = shape[1:]
        offset_path = os.path.join(self.tmp_folder, 'cc_offsets.json')
        dep = block_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                         input_path=self.input_path, input_key=self.input_key,
                         output_path=self.output_path, output_key=self.output_key,
                         threshold=self.threshold, threshold_mode=self.threshold_mode,
                         mask_path=self.mask_path, mask_key=self.mask_key, channel=self.channel,
                         fused=self.fused, dependency=self.dependency)
        dep = offset_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                          shape=shape, save_path=offset_path, dependency=dep)
        dep = face_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                        input_path=self.output_path, input_key=self.output_key,
                        offsets_path=offset_path, dependency=dep)
        dep = assignment_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                              output_path=self.output_path, output_key=self.assignment_key,
                              shape=shape, offset_path=offset_path, dependency=dep)
        dep = write_task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                         input_path=self.output_path, input_key=self.output_key,
                         output_path=self.output_path, output_key=self.output_key,
                         assignment_path=self.output_path, assignment_key=self.assignment_key,
                         identifier='thresholded_components', offset_path=offset_path,
                         dependency=dep)
        return dep

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'block_components': block_tasks.BlockComponentsLocal.default_task_config(),
                        'merge_offsets': offset_tasks.MergeOffsetsLocal.default_task_config(),
                        'block_faces': face_tasks.BlockFacesLocal.default_task_config(),
                        'merge_assignments': assignment_tasks.MergeAssignmentsLocal.default_task_config(),
                        'write': write_tasks.WriteLocal.default_task_config()})
        return configs


class ThresholdAndWatershedWorkflow(WorkflowBase):
    input_path = Parameter()
    input_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    assignment_key = Parameter()
    threshold = FloatParameter()
    threshold_mode = Parameter(default='greater')
    mask_path = Parameter(default='')
    mask_key = Parameter(default='')
    channel = Parameter(default=None)

    def requires(self):
        dep = ThresholdedComponentsWorkflow(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs,
                                            config_dir=self.config_dir, target=self.target,
                                            input_path=self.input_path, input_key=self.input_key,
                                            output_path=self.output_path, output_key=self.output_key,
                                            assignment_key=self.assignment_key, threshold=self.threshold,
                                            threshold_mode=self.threshold_mode, mask_path=self.mask_path,
                                            mask_key=self.mask_key, channel=self.channel,
                                            dependency=self.dependency)
        ws_task = getattr(ws_tasks, self._get_task_name('WatershedFromSeeds'))
        return ws_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                       dependency=dep, input_path=self.input_path, input_key=self.input_key,
                       seeds_path=self.output_path, seeds_key=self.output_key,
                       output_path=self.output_path, output_key=self.output_key,
                       mask_path=self.mask_path, mask_key=self.mask_key)

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'watershed_from_seeds': ws_tasks.WatershedFromSeedsLocal.default_task_config(),
                        **ThresholdedComponentsWorkflow.get_config()})
        return configs
